// dsort_tx.h -- the host transport's collectives of one sample sort (dsort_comm_init_transport):
// bounded waits and rank-symmetric failure.  Plain host C++ (no HIP): libdsort includes it, and so
// does the CPU test harness tests/tx/tx_harness.cpp, which runs this very sequencing over gloo.
//
// The reference's master learns of a dead worker from a socket error and carries on
// (server.c:358-395, 421-449).  The sample sort's host transport has the same duty towards its
// peers: every rank runs the same fixed sequence of collectives (key counts, samples, bucket
// starts, the key waves), and a rank that fails locally between two of them (an allocation, a HIP
// error, a stage the sort refuses) must not leave its peers blocked in a collective it never joins.
// So every collective, the first one included, is preceded by a GATE: an 8-byte all-gather of
// every rank's status.  A rank that failed reports its failure at the next gate and returns; every
// peer meets it there and returns DSORT_ECOMM naming that rank.  (ABI 5 gated the 2nd..last only,
// so a rank failing before its first collective -- the presorted entry's local staging, or a
// failure injected at collective 0 -- left its peers blocked in that collective: ADVICE r5.)  A callback that fails or gives up (the
// transport itself broke, or the exchange deadline passed) ends the sequence on that rank: no
// further collective runs on a broken transport.  The callbacks bound their own waits by
// dsort_comm_deadline_ms (the remainder of DSORT_OPT_COMM_TIMEOUT_MS), so a peer that hangs
// (never reaches a collective) surfaces as DSORT_ETIMEOUT on the others, not as a hang.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include <string>
#include <vector>

#include "dsort.h"

namespace dsort {

inline double tx_now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

class TxSeq {
  public:
    // t: the caller's transport over P ranks; deadline on the tx_now_ms() scale (0 = none); ncoll:
    // the collectives this sort will run (a gate sits in front of each).
    TxSeq(const dsort_transport &t, int P, double deadline, int ncoll)
        : t_(t), P_(P), deadline_(deadline), left_(ncoll) {}

    int allgather(const void *send, void *recv, size_t bytes, const char *what) {
        int rc = enter(what);
        if (rc) return rc;
        return done(t_.allgather(t_.user, send, recv, bytes), what);
    }
    int alltoallv(const void *send, const size_t *sc, const size_t *sd, void *recv, const size_t *rc_,
                  const size_t *rd, const char *what) {
        int rc = enter(what);
        if (rc) return rc;
        return done(t_.alltoallv(t_.user, send, sc, sd, recv, rc_, rd), what);
    }
    // more collectives in this sort (once the path is known: the bucket exchange or the merge path)
    void plan(int more) { left_ += more; }
    // This rank failed locally: tell the peers at the next gate (when a collective is still ahead
    // and the transport works), so that they leave the sequence there too.
    void report_failure(int code) {
        if (broken_ || left_ <= 0) return;
        int64_t st = code ? code : DSORT_ECOMM;
        std::vector<int64_t> all((size_t)P_);
        left_ = 0;  // (whatever the gate says: this rank runs no further collective)
        (void)call_gate(st, all.data(), "failure report");
    }
    // remaining milliseconds before the deadline (-1: none; 0: passed)
    int64_t remaining_ms() const {
        if (deadline_ <= 0) return -1;
        const double r = deadline_ - tx_now_ms();
        return r > 0 ? (int64_t)r + 1 : 0;
    }
    const std::string &error() const { return err_; }
    int failed_peer() const { return failed_peer_; }
    bool broken() const { return broken_; }
    int collectives_done() const { return started_; }

  private:
    int enter(const char *what) {
        if (broken_) return set(DSORT_ECOMM, std::string(what) + ": the host transport failed earlier");
        if (left_ <= 0) return set(DSORT_EINVAL, std::string(what) + ": more collectives than planned");
        if (deadline_ > 0 && tx_now_ms() > deadline_) {
            broken_ = true;
            return set(DSORT_ETIMEOUT, std::string(what) + ": the exchange deadline (DSORT_OPT_COMM_TIMEOUT_MS) passed");
        }
        {  // the gate in front of every collective
            std::vector<int64_t> all((size_t)P_);
            int rc = call_gate(0, all.data(), what);
            if (rc) return rc;
            for (int r = 0; r < P_; ++r)
                if (all[(size_t)r]) {
                    failed_peer_ = r;
                    left_ = 0;
                    return set(DSORT_ECOMM, std::string(what) + ": rank " + std::to_string(r) +
                                                " failed locally (error " + std::to_string(all[(size_t)r]) +
                                                ") and left the exchange");
                }
        }
        --left_;
        ++started_;
        return DSORT_OK;
    }
    int call_gate(int64_t st, int64_t *all, const char *what) {
        return done(t_.allgather(t_.user, &st, all, sizeof st), (std::string(what) + " (status gate)").c_str());
    }
    int done(int r, const char *what) {
        if (r == 0) return DSORT_OK;
        broken_ = true;
        left_ = 0;
        if (r == DSORT_ETIMEOUT)
            return set(DSORT_ETIMEOUT, std::string("host transport ") + what +
                                           ": no answer before the exchange deadline (DSORT_OPT_COMM_TIMEOUT_MS)");
        return set(DSORT_ECOMM, std::string("host transport ") + what + " failed (callback returned " +
                                    std::to_string(r) + ")");
    }
    int set(int code, const std::string &m) {
        err_ = m;
        return code;
    }

    dsort_transport t_;
    int P_;
    double deadline_;
    int left_;         // collectives still ahead
    int started_ = 0;  // collectives entered
    bool broken_ = false;
    int failed_peer_ = -1;
    std::string err_;
};

// Scope guard of a sample sort on the host transport: leaving the sort before its last collective
// (any error path) reports the failure at the next gate.
struct TxGuard {
    TxSeq *seq = nullptr;
    bool finished = false;
    int code = DSORT_ECOMM;
    ~TxGuard() {
        if (seq && !finished) seq->report_failure(code);
    }
};

}  // namespace dsort
