// tx_harness.cpp -- TEST HARNESS (not product code): the host transport's collective sequence of
// the bucket exchange (csrc/dsort_tx.h, the same TxSeq / TxGuard libdsort's sample sort runs) on
// the CPU, with synthetic payloads in place of the GPU's keys, so that tests/test_tx_gates.py can
// check over gloo (world size 3, no GPU) that a rank failing locally -- or hanging -- between two
// collectives makes every rank return within the exchange deadline instead of blocking.
//
// The sequence is sample_sort + sample_sort_bx's (dsort_api.hip) on the host transport: [gate]
// key-count all-gather, [gate] sample all-gather, [gate] bucket-start all-gather, [gate] key
// all-to-all of wave 0, [gate] wave 1.
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "dsort_tx.h"

namespace {
dsort::TxSeq *g_seq = nullptr;
}

extern "C" {

// Milliseconds left before the running sequence's deadline (-1: none), as dsort_comm_deadline_ms.
int64_t txh_deadline_ms(void) { return g_seq ? g_seq->remaining_ms() : -1; }

// Runs the sequence on rank `me` of P.  Rank `fail_rank` fails locally right before collective
// `fail_at` (returns DSORT_EHIP through the guard, as any local error of the library does), or,
// with hang_ms > 0, stalls that long there first.  Returns the sequence's result; msg gets the
// error text; *peer = the failed rank a gate reported (-1 none); *ncoll = collectives entered.
int txh_run(const dsort_transport *t, int P, int me, int waves, int fail_rank, int fail_at, int hang_ms,
            int64_t timeout_ms, char *msg, size_t cap, int *peer, int *ncoll) {
    const double deadline = timeout_ms > 0 ? dsort::tx_now_ms() + (double)timeout_ms : 0.0;
    dsort::TxSeq seq(*t, P, deadline, 1);
    g_seq = &seq;
    int rc = DSORT_OK;
    std::string err;
    {
        dsort::TxGuard guard;
        guard.seq = &seq;
        int k = 0;  // collectives entered so far on the normal path
        auto local_step = [&]() -> int {
            if (me != fail_rank || k != fail_at) return DSORT_OK;
            if (hang_ms > 0) {
                usleep((useconds_t)hang_ms * 1000u);
                return DSORT_OK;
            }
            err = "injected local failure before collective " + std::to_string(k);
            return DSORT_EHIP;
        };
        auto wrap = [&](int r) -> int {
            if (r) err = seq.error();
            ++k;
            return r;
        };
        // 0. key counts (8 bytes per rank)
        const uint64_t nl = 1000 + (uint64_t)me;
        std::vector<uint64_t> counts((size_t)P);
        if (!rc) rc = local_step();
        if (!rc) rc = wrap(seq.allgather(&nl, counts.data(), 8, "key count all-gather"));
        if (!rc) seq.plan(2 + waves);
        // 1. samples (64 bytes per rank)
        std::vector<uint8_t> smp(64, (uint8_t)me), all((size_t)64 * P);
        if (!rc) rc = local_step();
        if (!rc) rc = wrap(seq.allgather(smp.data(), all.data(), smp.size(), "samples all-gather"));
        // 2. bucket starts
        std::vector<uint64_t> hb(5, (uint64_t)me), hb_all((size_t)5 * P);
        if (!rc) rc = local_step();
        if (!rc) rc = wrap(seq.allgather(hb.data(), hb_all.data(), 40, "bucket starts all-gather"));
        // 3.. the key waves: 4 bytes to every rank
        for (int w = 0; w < waves && !rc; ++w) {
            std::vector<uint8_t> snd((size_t)4 * P, (uint8_t)(16 * w + me)), rcv((size_t)4 * P);
            std::vector<size_t> sc((size_t)P, 4), sd((size_t)P), rcn((size_t)P, 4), rd((size_t)P);
            for (int q = 0; q < P; ++q) sd[(size_t)q] = rd[(size_t)q] = (size_t)4 * q;
            rc = local_step();
            if (!rc)
                rc = wrap(seq.alltoallv(snd.data(), sc.data(), sd.data(), rcv.data(), rcn.data(), rd.data(),
                                        w ? "key all-to-all (wave 1)" : "key all-to-all (wave 0)"));
            for (int q = 0; q < P && !rc; ++q)
                if (rcv[(size_t)4 * q] != (uint8_t)(16 * w + q)) {
                    err = "wave payload mismatch";
                    rc = DSORT_EINVAL;
                }
        }
        if (!rc) guard.finished = true;
        guard.code = rc ? rc : DSORT_ECOMM;
    }  // (the guard reports a local failure at the next gate here)
    if (peer) *peer = seq.failed_peer();
    if (ncoll) *ncoll = seq.collectives_done();
    g_seq = nullptr;
    if (msg && cap) {
        strncpy(msg, err.c_str(), cap - 1);
        msg[cap - 1] = 0;
    }
    return rc;
}

}  // extern "C"
