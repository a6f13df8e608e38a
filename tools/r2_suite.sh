#!/bin/bash
# the whole GPU suite (verbose summary of failures)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_suite.log 2>&1
rc=$?; tail -4 gpurun_out/tests_suite.log; exit $rc
