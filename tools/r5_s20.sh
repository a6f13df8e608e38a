export OUT=gpurun_out/r5_s20
STEPS="pmclat" PMC_MATCH="gram|lo_resid|lo_fold|lo_approx" bash tools/r5.sh
