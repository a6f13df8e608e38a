// summary.h -- what the host replay needs of one scored block of slots
// (device-side candidate selection, summary.hip).
//
// GCRANSAC::run (GCRANSAC.h:286-531) acts on a hypothesis only when it is a
// strict new best with a valid model (:440-446); max_iteration changes only
// then (:479-483, getIterationNumber :738-757) and LO runs only then
// (:467-477).  Every other hypothesis is iteration accounting (:293-339) plus
// the inlier-buffer write of the last one processed (:460).  So a block of
// slots is summarised by
//   - its prefix-maximum chain: the hypotheses whose finished MSAC score beats
//     every earlier valid one of the block and a bar (the best known when the
//     block was summarised).  Every strict new best of the replay is one of
//     them, whatever LO does in between (LO only raises the bar).  A
//     hypothesis with flagged decisions (exact.h: its score in the reference's
//     arithmetic is only known after the host's recheck) is always a member
//     and never raises the running maximum, so the chain still holds every
//     possible new best;
//   - the iteration and hypothesis totals, and for each chain member the
//     iterations and hypotheses before it (prefix sums of inc);
//   - the block's last live hypothesis (the buffer the replay holds at a
//     chunk boundary), and on request (locate) the slot where a given
//     iteration count is reached and the last live hypothesis before it.
// Blocks are per chunk and rank: one rank's block is all a single-GPU run
// needs; a hypothesis-sharded run all-gathers these fixed-size records
//  instead of per-hypothesis data.
#pragma once

#include <cstdint>

namespace gcr {

constexpr int kCandCap = 32;           // chain members per summary (more: overflow + continuation)

struct SumHyp {                        // one hypothesis of a block
    uint32_t pos;                      // position slot * per + q in the block
    uint32_t inc;                      // its slot's inc (1 .. 102)
    uint64_t it_before;                // sum of inc over the block's slots before its slot
    uint64_t hyps_before;              // live hypotheses before it in the block
    uint32_t n0, n1;                   // raw MSAC accumulators (ScoreOut)
    uint32_t fl;                       // flagged MSAC decisions (exact.h): the host rechecks them
    uint32_t lfl;                      // flagged list decisions (small-scored chunks with list bits)
    double v0, v1, tot;
    double m[9];                       // the model (RectModel: 7 doubles, GeoModel: 9)
};

struct BlockSummary {
    uint64_t inc_total;                // sum of inc over the block
    uint64_t hyps_total;               // live hypotheses of the block
    uint32_t ncand;                    // chain members in cand[]
    uint32_t overflow;                 // more members exist after cand[ncand - 1]
    uint32_t has_last;                 // `last` is set
    uint32_t stop_found;               // locate: the block reaches the iteration target
    uint64_t stop_slot;                // locate: first slot whose iterations-before reach it
    uint64_t stop_it_before;           //   its iterations before (block-relative)
    uint64_t stop_hyps_before;         //   live hypotheses before it (block-relative)
    uint32_t resume_pos;               // overflow: continue the chain from this position
    uint32_t pad;
    double resume_bar;                 //   with this bar
    SumHyp last;                       // last live hypothesis (of the block / before stop_slot)
    SumHyp cand[kCandCap];
};

}  // namespace gcr
