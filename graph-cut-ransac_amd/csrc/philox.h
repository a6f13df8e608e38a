// philox.h -- counter-based sampler that replaces the reference's per-sample
// std::random_device + std::mt19937 + full std::shuffle (GCRANSAC.h:53-80).
//
// The reference draws each minimal sample as the first m entries of a uniformly
// shuffled copy of the index pool, i.e. a uniform *ordered* m-subset.  Here the
// same distribution is produced in O(m) by rejection of repeated indices, with
// every random word addressed by (seed, index, sub, stream, class, block) so any
// outer-iteration slot can be drawn independently on any lane of any GPU.
//
// Key/counter layout (identical in the CPU oracle, oracle/gcr_oracle.cpp):
//   key  = {seed[31:0], seed[63:32]}
//   ctr  = {index[31:0], index[63:32], sub, stream<<24 | class<<16 | block}
//   main loop : index = outer-iteration slot, sub = attempt (0..100), stream 0
//   local opt.: index = graph-cut round id,   sub = trial,             stream 1
// Each Philox4x32-10 block yields two 64-bit words; word w lives in block w/2.
// A draw is mulhi64(word, n) (bias < n / 2^64).
#pragma once

#include "gcr_hd.h"

namespace gcr {

enum : uint32_t { kStreamMain = 0, kStreamLO = 1 };
constexpr uint32_t kMaxSampleDraws = 4096;   // termination guard, never reached in practice

GCR_HD void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        const uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

GCR_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * (unsigned __int128)b) >> 64);
#endif
}

// Stream of 64-bit words for one (seed, index, sub, stream, class) address.
struct WordStream {
    uint32_t key[2];
    uint32_t ctr[4];
    uint32_t buf[4];
    uint32_t next;   // next word index

    GCR_HD WordStream(uint64_t seed, uint64_t index, uint32_t sub, uint32_t stream, uint32_t cls) {
        key[0] = (uint32_t)seed;
        key[1] = (uint32_t)(seed >> 32);
        ctr[0] = (uint32_t)index;
        ctr[1] = (uint32_t)(index >> 32);
        ctr[2] = sub;
        ctr[3] = (stream << 24) | ((cls & 0xffu) << 16);
        next = 0;
        buf[0] = buf[1] = buf[2] = buf[3] = 0;
    }
    GCR_HD uint64_t word() {
        const uint32_t w = next++;
        if ((w & 1u) == 0) {
            uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3] | ((w >> 1) & 0xffffu)};
            philox4x32_10(c, key, buf);
            return (uint64_t)buf[0] | ((uint64_t)buf[1] << 32);
        }
        return (uint64_t)buf[2] | ((uint64_t)buf[3] << 32);
    }
};

// Draws m distinct values uniformly from [0, n), in draw order, into out[0..m).
// Returns false only if the draw budget is exhausted (n < m, or astronomically
// unlikely for n >= m).
template <int MAXM>
GCR_HD bool sample_distinct(WordStream& ws, uint64_t n, int m, uint32_t* out) {
    int j = 0;
    while (j < m) {
        if (ws.next >= kMaxSampleDraws) return false;
        const uint32_t v = (uint32_t)mulhi64(ws.word(), n);
        bool dup = false;
#pragma unroll
        for (int q = 0; q < MAXM; ++q)
            if (q < j && out[q] == v) dup = true;
        // constant-index stores: on the device out[] stays in registers (a
        // dynamic out[j] put the caller's index array in LDS / scratch)
#pragma unroll
        for (int q = 0; q < MAXM; ++q)
            if (!dup && q == j) out[q] = v;
        j += dup ? 0 : 1;
    }
    return true;
}

}  // namespace gcr
