/* ss.h -- control protocol of the multi-GPU sample sort driven from C
 * (dsort_master --mode samplesort / dsort_worker --mode samplesort).
 *
 * Roles follow the reference: the master (server.c) owns the input and its chunk replicas and
 * hands one equal contiguous chunk to every worker (server.c:185-216); a worker (client.c) is one
 * process per GPU.  What changes for the multi-GPU path:
 *   - the chunk replicas live in a POSIX shared-memory segment the master creates
 *     (/dev/shm/dsort-ss-<pid>); every worker maps it and pins it (dsort_host_register), so a
 *     worker's chunk and, after a failure, a dead worker's chunk move host -> HBM by DMA;
 *   - the single-master gather (server.c:414-415) becomes the sample sort's all-to-all between
 *     the workers (libdsort, RCCL over xGMI; or the "relay" transport through the master when
 *     the workers share one GPU or RCCL is unusable);
 *   - a failed worker (socket EOF, process exit, or no heartbeat within --timeout-ms) is replaced
 *     by the reference's rule (server.c:368-384): its chunk goes to the first live worker
 *     (first-live) or to the next live one (next-live); the survivors abort the communicator,
 *     build a new one (new RCCL unique id from the master), the assignee sorts the dead chunk from
 *     the pinned replica and merges it into its own run, and the exchange runs again over the
 *     survivors.  The output is the concatenation of the survivors' slices in their new rank order.
 *
 * Framing: wire.h v1 headers (24 bytes) with elem_bytes = 1 and count = payload bytes; `status`
 * carries the relay sequence number.  All structs are native-endian (one host). */
#ifndef DSORT_SS_H
#define DSORT_SS_H

#include <stdint.h>

enum ss_type {
    SS_HELLO = 32,      /* worker -> master: ss_hello                                       */
    SS_JOB = 33,        /* master -> worker: ss_job                                         */
    SS_READY = 34,      /* worker -> master: ss_ready (chunk staged, communicator up)       */
    SS_GO = 35,         /* master -> worker: start the timed sort                           */
    SS_DONE = 36,       /* worker -> master: ss_done (one epoch's exchange finished)        */
    SS_PLAN = 37,       /* master -> worker: ss_plan (recovery epoch after a failure)       */
    SS_BYE = 38,        /* master -> worker: exit                                           */
    SS_HB = 39,         /* worker -> master: heartbeat                                      */
    SS_RELAY_AG = 40,   /* worker -> master: all-gather contribution (relay transport)      */
    SS_RELAY_A2A = 41,  /* worker -> master: all-to-all-v pieces (relay transport)          */
    SS_RELAY_RESP = 42, /* master -> worker: the relayed result                             */
    SS_GET_SLICE = 43,  /* master -> worker: send the sorted slice (--output)               */
    SS_SLICE = 44,      /* worker -> master: the slice's keys                               */
};

#define SS_MAX_WORKERS 64
#define SS_MAX_CHUNKS 64

typedef struct ss_hello {
    int32_t pid;
    int32_t device;
} ss_hello;

typedef struct ss_job {
    uint32_t epoch, world, rank, key_bytes; /* key_bytes 4 (int32) or 8 (int64)           */
    uint64_t n_total;
    uint64_t chunk_off, chunk_len;          /* this rank's chunk, in keys                     */
    uint64_t seed;
    uint32_t transport;                     /* 0 rccl, 1 relay through the master             */
    uint32_t source;                        /* 0 uniform, 1 zipf (worker generates its chunk
                                               into the replica), 2 replica already filled   */
    int32_t kill_after_pass;                /* fault injection: DSORT_OPT_KILL_AFTER_STAGE, -1 off */
    int32_t kill_in_exchange;               /* -1 off, 1 / 2 = DSORT_OPT_KILL_IN_EXCHANGE     */
    int64_t comm_timeout_ms;
    uint32_t heartbeat_ms;
    int32_t kill_in_recovery;               /* fault injection: 1 = die on the first recovery PLAN
                                               (a second failure while the survivors rebuild)   */
    int32_t hang_before_exchange;           /* fault injection: 1 = SIGSTOP itself after the local
                                               sort (a hung, not dead, worker: only silence and
                                               the peers' failed exchanges show it)            */
    char shm_name[64];
    char uid[128];                          /* RCCL unique id of this epoch                   */
} ss_job;

typedef struct ss_ready {
    uint32_t rank, pad;
    uint64_t n, fp_sum, fp_xor;             /* fingerprint of the chunk as staged             */
    double t_setup_ms;
} ss_ready;

typedef struct ss_done {
    uint32_t epoch, rank;
    int32_t status;                          /* 0 ok, else the DSORT_E* code of the exchange   */
    uint32_t pad;
    uint64_t n_out, descents, fp_sum, fp_xor, run_keys;
    int64_t first, last;
    double t_local_sort_ms;                  /* from GO to the end of the local sort           */
    double t_exchange_ms;                    /* the epoch's exchange + merge                   */
    double t_rebuild_ms;                     /* recovery: sorting + merging the extra chunks   */
} ss_done;

typedef struct ss_plan {
    uint32_t epoch, world, rank, nchunks;    /* nchunks: chunks this survivor owns from now   */
    uint32_t chunks[SS_MAX_CHUNKS];          /* original chunk indices (its own included)      */
    char uid[128];
} ss_plan;

#endif
