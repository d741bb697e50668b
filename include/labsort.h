/*
 * include/labsort.h -- C-ABI of liblabsort.so, the MI355X-native (gfx950) sort.
 *
 * Plain pointers and sizes only (no HIP or torch types): `stream` is a
 * hipStream_t passed as void* (NULL = the null stream), device pointers come
 * from hipMalloc / torch tensors.  Every function returns a LABSORT_* status.
 *
 * What each entry replaces in the reference (`Sord Radix y Merge/`):
 *   labsort_sort_host      order_array(int*, int)               lab.cu:303-402, lab.h:9
 *                          (host pointer in, sorted in place, synchronous)
 *   labsort_sort_device    stages 1-3 of order_array between the H2D copy
 *                          (lab.cu:321) and the D2H copy (lab.cu:397)
 *   labsort_wave_tile_sort radix_sort_kernel (lab.cu:47-87): per-tile bit
 *                          split with early exit, wave64 tiles instead of warp32
 *   labsort_tile_sort      stage 1+2 of order_array (lab.cu:323-346): sorted
 *                          runs of labsort_tile_keys() keys
 *   labsort_merge_pass     stage 3 iteration (separators_kernel +
 *                          merge_segments_kernel, lab.cu:358-391)
 *   labsort_merge          deviceOrderedJoin (lab.cu:144-182) generalised to a
 *                          diagonal range of merge(A,B); used by the multi-GPU
 *                          merge-split exchange
 *   labsort_histogram      the global digit count of letra.pdf's split (no
 *                          counterpart kernel in lab.cu)
 *   sort(int*, int)        the north_star's name for order_array
 * The C++-linkage drop-ins order_array / order_with_trust live in lab.h.
 */
#ifndef LABSORT_H
#define LABSORT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define LABSORT_OK 0
#define LABSORT_ERR_ARG 1        /* bad argument (NULL, n too large, workspace too small) */
#define LABSORT_ERR_HIP 2        /* a HIP runtime call failed: labsort_last_hip_error() */
#define LABSORT_ERR_DEVICE 3     /* a kernel reported an internal error (bounded spin expired) */
#define LABSORT_ERR_PEER 4       /* distributed sort: another rank failed (this one gave up with it) */

/* algorithms */
#define LABSORT_ALGO_RADIX 0     /* LSD radix, 8-bit digits: gathered passes for 2^16 <= n < 2^25,
                                    onesweep scatter passes outside (LABSORT_RADIX_IMPL=onesweep or
                                    =gather forces one) */
#define LABSORT_ALGO_MERGE 1     /* LDS tile radix + merge-path merge passes */
#define LABSORT_ALGO_RADIX1 2    /* LSD radix with 1-bit digits: letra.pdf's split, 32 passes */
#define LABSORT_ALGO_AUTO 3      /* MERGE for n <= LABSORT_AUTO_MERGE_MAX_KEYS (fewer launches and
                                    less fixed cost at small n) and above the radix limit
                                    (labsort_max_keys(RADIX), e.g. 2^30 keys), RADIX between; the
                                    default of the host drop-ins order_array / sort (LABSORT_ALGO
                                    env overrides) */
#define LABSORT_AUTO_MERGE_MAX_KEYS (1u << 16) /* r27: the fused gathered radix wins from ~1.5 x 2^16 */
/* key/value sorts (labsort_sort_pairs_device, AUTO): merge up to here.  Their radix has no
   fused small path (histogram, plan and four persistent passes at every size), so they keep
   the r19 crossover measured before the keys-only threshold moved */
#define LABSORT_AUTO_PAIRS_MERGE_MAX_KEYS (1u << 18)

/* key types: how the 32-bit words are ordered */
#define LABSORT_KEY_U32 0
#define LABSORT_KEY_I32 1

/* generator distributions (oracle/cpu_sort.cpp uses the same codes and formula) */
#define LABSORT_DIST_U32 0
#define LABSORT_DIST_U31 1
#define LABSORT_DIST_MOD100 2
#define LABSORT_DIST_MOD1000 3
#define LABSORT_DIST_SORTED 4
#define LABSORT_DIST_REVERSED 5
#define LABSORT_DIST_CONST 6
#define LABSORT_DIST_LOWBITS 7

/* kernel classes for the timing hooks */
#define LABSORT_K_HISTOGRAM 0
#define LABSORT_K_ONESWEEP 1
#define LABSORT_K_TILE_SORT 2
#define LABSORT_K_MERGE 3
#define LABSORT_K_PARTITION 4
#define LABSORT_K_GSWEEP 5       /* gathered radix pass (LABSORT_ALGO_RADIX, 2^16 <= n < 2^25) */
#define LABSORT_K_GCOPY 6        /* its final gathered copy */
#define LABSORT_K_COPY 7         /* the streaming copy (labsort_copy: the bench's copy ceiling) */
#define LABSORT_K_MERGE4 8       /* four-way merge pass of the merge sort (k_m4_rank + k_m4_merge) */
#define LABSORT_K_COUNT 9

/* ---- library info ---- */
const char *labsort_version(void);
const char *labsort_error_string(int status);
int labsort_last_hip_error(void);                 /* hipError_t of the last failure */
const char *labsort_hip_error_string(int hip_error);
size_t labsort_max_keys(int algo);                /* largest n a device sort accepts */
size_t labsort_tile_keys(void);                   /* run length produced by labsort_tile_sort */
size_t labsort_merge_tile_keys(void);             /* output keys per merge workgroup */

/* ---- whole sorts ---- */
/* Bytes of device workspace labsort_sort_device needs for n keys. */
size_t labsort_workspace_bytes(size_t n, int algo);
/* Sort n keys from d_in into d_out (d_in == d_out allowed: in place).
 * Asynchronous on `stream`; no host synchronisation, graph-capturable. */
int labsort_sort_device(const void *d_in, void *d_out, size_t n, int key_type, int algo, void *d_workspace,
                        size_t workspace_bytes, void *stream);
/* Host pointer in/out, synchronous: the order_array contract (lab.cu:303).
 * From 2^27 keys the copies are pipelined: 8 chunks copied H2D while earlier chunks
 * sort (each by `algo` resolved at the chunk's size), two half merges, and the final
 * merge by 8 diagonal ranges whose D2H copies start as each range lands
 * (LABSORT_HOST_PIPE=0 turns it off, =1 forces it from 2^16 keys).
 * Returns LABSORT_ERR_DEVICE when a kernel reported an internal error. */
int labsort_sort_host(void *h_keys, size_t n, int key_type, int algo);
/* Device-side status of the last labsort_sort_device(n, algo) that used d_workspace:
 * synchronises `stream`, then returns LABSORT_ERR_DEVICE if a kernel of that sort set
 * the workspace's error word (radix: a bounded look-back spin expired; merge: a four-way
 * block whose cuts were inconsistent was skipped -- the result is not valid), else
 * LABSORT_OK.  The error word is the first 32-bit word of the workspace, cleared at the
 * start of every sort longer than one tile (one tile: no error word, LABSORT_OK).  The
 * reference's policy (CUDA_CHK after every launch, utils.h:18-26) checks launch status
 * only; this adds the kernels' own failure report. */
int labsort_workspace_status(const void *d_workspace, size_t n, int algo, void *stream);
/* The same for the last labsort_sort_pairs_device(n, algo) on d_workspace. */
int labsort_pairs_workspace_status(const void *d_workspace, size_t n, int algo, void *stream);

/* ---- the merge-sort path across GPUs (the reference
 * is single-GPU, lab.cu:303-402).  One schedule (csrc/dist_plan.h) for every form:
 * each rank sorts its shard locally (LABSORT_ALGO_AUTO), the ranks agree on p-1
 * (key, rank, position) splitters from a regular sample of every sorted shard, cut
 * their shards at them (labsort_upper_bound), send piece j to rank j by pairwise
 * send/recv with every peer at once, and merge the p received runs in rank order
 * (labsort_merge_runs pair passes, then the last level by diagonal ranges).  Rank r
 * ends with the contiguous range [goff, goff + count) of the sorted array. ----
 *
 * One process, several GPUs (one host thread per rank): sort a host buffer in place.
 * Rank r copies the shard h_keys[r*n/p, (r+1)*n/p) over its own PCIe link in 8 chunks
 * while earlier chunks sort (from 2^24 keys per rank; LABSORT_HOST_PIPE=0 never, =1
 * from 2^16), and copies its merged range back to its global offset range by range as
 * the last merge level lands.  LABSORT_PIN=1 page-locks the caller's array for the
 * call (hipHostRegister).  transport: LABSORT_XFER_PEER (hipMemcpyPeerAsync into each
 * receiver's slot; ranks may share a device), LABSORT_XFER_RCCL (ncclSend/ncclRecv
 * with every peer in one group per rank, communicators from ncclCommInitAll; one rank
 * per device) or LABSORT_XFER_AUTO (= PEER).  Synchronous.  order_array / sort use
 * labsort_sort_host_multi when LABSORT_GPUS > 1. */
#define LABSORT_XFER_AUTO 0
#define LABSORT_XFER_RCCL 1
#define LABSORT_XFER_PEER 2
#define LABSORT_MULTI_MAX_RANKS 8
/* phases of labsort_multi_timing / labsort_dist_timing, ms of the last call (device
 * timeline, max over ranks; phases may overlap): 0 H2D (host input), 1 local sort,
 * 2 plan (samples + splitters + cut points, collectives included), 3 exchange, 4 merge,
 * 5 D2H tail after the merge (host output), 6 total (host wall time), 7 the plan's own
 * work (host clock: from the rank's local sort seen complete to the plan's end, minus
 * the time spent inside its collectives), 8 the plan's wait (time inside the
 * collectives: mostly waiting for the slowest rank to arrive) */
#define LABSORT_MULTI_PHASES 9
/* Collectives of one schedule call, in order: 0 samples (allgather), 1 piece counts
 * (allgather), 2 buffer growth (allgather; runs only when a range outgrew the pre-sized
 * receive buffer).  labsort_multi_collectives / labsort_dist_collectives: host wall clock
 * (ms since the rank's call started) at which each rank arrived at / returned from each
 * of them in the last call (-1: did not run); arrive[r * ncoll + k], leave[r * ncoll + k]. */
#define LABSORT_MULTI_COLLECTIVES 3
int labsort_sort_host_multi(void *h_keys, size_t n, int key_type, int ngpus);  /* devices 0..ngpus-1 */
int labsort_sort_host_ranks(void *h_keys, size_t n, int key_type, int nranks, const int *devices, int transport);
int labsort_multi_timing(double *phase_ms, int nphases, size_t *max_sent_bytes);
int labsort_multi_collectives(double *arrive, double *leave, int nranks, int ncoll);
int labsort_multi_last_hip_error(void);
/* keys of each rank's range of the sorted array in the last call (ranks in order) */
int labsort_multi_range_counts(size_t *counts, int nranks);
/* text of the last failure of a multi-GPU call (HIP call, RCCL result, callback) */
const char *labsort_multi_error_detail(void);
/* The exchange plan alone, on host shards (sorted h_shards[r][0..m[r]) per rank;
 * std::upper_bound stands in for the device bound queries): writes the cut points,
 * h_cuts[r*(nranks+1) + j] = first position of the piece rank r sends to rank j.
 * Test hook for the schedule; no GPU involved. */
int labsort_multi_plan(const uint32_t *const *h_shards, const size_t *m, int nranks, int key_type, size_t *h_cuts);

/* One process per GPU (torch.distributed.run / mpirun style): a communicator handle
 * per rank, then one labsort_dist_sort call per rank and sort.
 *   RCCL: rank 0 calls labsort_comm_unique_id, the id (LABSORT_COMM_ID_BYTES) is
 *         broadcast by the caller's own means, every rank calls labsort_comm_init_rccl
 *         with its device current (ncclCommInitRank).
 *   Host callbacks: the collectives are the caller's (labsort_host_coll over host
 *         buffers; device pieces are staged): several ranks may share a GPU (tests).
 * A rank whose own step fails (local sort, samples, bounds, buffers) still reports its
 * status in every collective up to the exchange, so every rank returns an error together
 * (the failed one its own, the others LABSORT_ERR_PEER) instead of waiting for it. */
#define LABSORT_COMM_ID_BYTES 128
/* ranks of one communicator: the receive-side merge takes two halves of at most 8 runs */
#define LABSORT_DIST_MAX_RANKS 16
typedef struct labsort_comm *labsort_comm_t;
typedef struct {
    void *ctx;
    /* h_out[i * bytes .. (i+1) * bytes) = rank i's h_in; return 0 on success */
    int (*allgather)(void *ctx, const void *h_in, void *h_out, size_t bytes);
    /* send_bytes[j] bytes of h_send (pieces back to back in rank order) to rank j,
     * recv_bytes[i] bytes from rank i into h_recv (rank order); own entries are 0 */
    int (*alltoallv)(void *ctx, const void *h_send, const size_t *send_bytes, void *h_recv,
                     const size_t *recv_bytes);
} labsort_host_coll;
int labsort_comm_unique_id(void *id);
/* RCCL communicators are nonblocking (ncclConfig_t blocking = 0): every wait on the peers
 * -- the communicator's creation, each collective, the exchange -- polls
 * ncclCommGetAsyncError and ends at a deadline (LABSORT_COMM_TIMEOUT_S by default).  A
 * rank whose peer never arrives (its transport broke, it left) then returns
 * LABSORT_ERR_PEER and its communicator is aborted (ncclCommAbort: its kernels and proxy
 * stop); later sorts on an aborted communicator return LABSORT_ERR_PEER at once. */
#define LABSORT_COMM_TIMEOUT_S 120.0
int labsort_comm_init_rccl(labsort_comm_t *comm, const void *id, int nranks, int rank);
/* the deadline of every wait on the peers: of `comm`, or (comm NULL) of the in-process
 * ranks' RCCL transport and of the communicators created afterwards */
int labsort_comm_set_timeout(labsort_comm_t comm, double seconds);
int labsort_comm_init_host(labsort_comm_t *comm, int nranks, int rank, const labsort_host_coll *coll);
int labsort_comm_destroy(labsort_comm_t comm);
/* This rank's shard d_keys[0..m) (device, on the comm's device; left untouched) in;
 * out: *d_result = this rank's range of the sorted array (*count keys, global offset
 * *global_offset), in a buffer the communicator owns until its next sort.  Runs on
 * `stream` (ordered after the work already queued there) and returns once the range
 * is complete. */
int labsort_dist_sort(labsort_comm_t comm, const void *d_keys, size_t m, int key_type, void *stream,
                      const void **d_result, size_t *count, size_t *global_offset);
int labsort_dist_timing(labsort_comm_t comm, double *phase_ms, int nphases, size_t *sent_bytes);
/* this rank's arrival / return times at the collectives of its last sort (ncoll entries) */
int labsort_dist_collectives(labsort_comm_t comm, double *arrive, double *leave, int ncoll);
int labsort_dist_last_hip_error(labsort_comm_t comm);
/* TEST HOOK of the multi-GPU schedule (tests only; the product never arms it): rank
 * `rank` of the following labsort_dist_sort / labsort_sort_host_ranks calls fails at
 * `phase` -- "local_sort", "bounds", "recv", "grow" (the receive buffer's growth round) or
 * "exchange" (it leaves without taking part: a broken transport) -- as an out-of-memory
 * or an expired device spin would.  phase NULL disarms; an unknown phase is
 * LABSORT_ERR_ARG.  Process-wide. */
int labsort_test_fault(const char *phase, int rank);

/* ---- key/value (sort_by_key; no lab.cu counterpart, the reference sorts
 * keys only) ----
 * Stable sort of n (key, 4-byte payload) pairs: d_keys_in/d_vals_in -> d_keys_out/
 * d_vals_out (out-of-place or fully in place: keys_in == keys_out and vals_in ==
 * vals_out).  Equal keys keep their input order, so sorting (key, index) pairs gives a
 * stable argsort, from which payloads of any width can be gathered.
 * algo: LABSORT_ALGO_RADIX (8-bit LSD onesweep passes carrying the payload),
 * LABSORT_ALGO_MERGE (LDS tile sort of labsort_pair_tile_keys() pairs + merge-path
 * passes) or LABSORT_ALGO_AUTO (merge up to LABSORT_AUTO_PAIRS_MERGE_MAX_KEYS, radix above).
 * Asynchronous on `stream`, no allocation; d_ws >= labsort_pairs_workspace_bytes(n, algo). */
size_t labsort_pair_tile_keys(void);
size_t labsort_pairs_workspace_bytes(size_t n, int algo);
int labsort_sort_pairs_device(const void *d_keys_in, const void *d_vals_in, void *d_keys_out, void *d_vals_out,
                              size_t n, int key_type, int algo, void *d_workspace, size_t workspace_bytes,
                              void *stream);

/* ---- building blocks (exposed for tests and the multi-GPU driver) ---- */
/* Sort every 64-key tile of d_keys in place by 1-bit splits (ballot + mbcnt +
 * ds_permute), stopping early once the tile is sorted: radix_sort_kernel's job. */
int labsort_wave_tile_sort(void *d_keys, size_t n, int key_type, void *stream);
/* Sort every labsort_tile_keys() tile of d_in into d_out (in place allowed). */
int labsort_tile_sort(const void *d_in, void *d_out, size_t n, int key_type, void *stream);
/* One merge pass: runs of `run` keys (power of two, >= labsort_merge_tile_keys()/2)
 * pairwise merged into runs of 2*run.  d_part: >= labsort_merge_parts(n) words. */
size_t labsort_merge_parts(size_t n);
int labsort_merge_pass(const void *d_in, void *d_out, size_t n, size_t run, int key_type, uint32_t *d_part,
                       void *stream);
/* out[0 .. d1-d0) = elements d0 .. d1-1 of merge(A, B) (A before B on ties).
 * d_part: >= labsort_merge_parts(d1-d0) words. */
int labsort_merge(const void *d_a, size_t la, const void *d_b, size_t lb, void *d_out, size_t d0, size_t d1,
                  int key_type, uint32_t *d_part, void *stream);
/* Merge of up to 8 sorted runs lying back to back in d_in: run q =
 * d_in[h_offsets[q] .. h_offsets[q+1]), q < nruns (host array of nruns+1 offsets).
 * Writes the merged keys to d_out[h_offsets[0] .. h_offsets[nruns]) (d_out != d_in);
 * equal keys keep run order (stable): ceil(log2 nruns) levels of pairwise merge-path
 * passes over explicit pairs of runs (k_merge_pass_p, one launch per pair),
 * ping-ponging through the workspace so the last level writes d_out.  Generalises
 * separators_kernel + merge_segments_kernel (lab.cu:209-300) from 2 to K runs; the
 * multi-GPU schedule merges the runs a rank receives with it.
 * d_ws: >= labsort_merge_runs_workspace_bytes(h_offsets[nruns]) (ping-pong keys). */
size_t labsort_merge_runs_workspace_bytes(size_t n);
int labsort_merge_runs(const void *d_in, void *d_out, const size_t *h_offsets, int nruns, int key_type,
                       void *d_workspace, size_t ws_bytes, void *stream);
/* d_hist[p * 2^bits + digit] += count of keys with that digit in pass p
 * (p = 0 .. ceil(32/bits)-1); bits = 8 or 1.  d_hist must be zeroed by the caller. */
int labsort_histogram(const void *d_keys, size_t n, int key_type, int bits, uint32_t *d_hist, void *stream);

/* d_out[i] = number of keys <= d_values[i] in the sorted run d_sorted[0..n) (key order):
 * the cut points of a rank's sorted shard at the common splitters of the multi-GPU
 * exchange (no lab.cu counterpart: the reference is single-GPU). */
int labsort_upper_bound(const void *d_sorted, size_t n, int key_type, const uint32_t *d_values, size_t nv,
                        uint32_t *d_out, void *stream);

/* ---- utilities ---- */
/* Counter-based generator, identical to oracle_fill: keys first..first+n-1. */
int labsort_fill(void *d_out, size_t n, uint64_t seed, int dist, uint64_t param, uint64_t first, void *stream);
/* d_out[0..n) = d_in[0..n) (32-bit words): a streaming copy with 16-B nontemporal loads and
 * stores in 16384-word tiles, one 1024-thread workgroup per CU -- the practical HBM rate of
 * a read-once / write-once pass, which bench.py reports beside each kernel's roofline. */
int labsort_copy(const void *d_in, void *d_out, size_t n, void *stream);
/* *d_count += number of i with key[i] > key[i+1] (0 = sorted). */
int labsort_count_descents(const void *d_keys, size_t n, int key_type, uint32_t *d_count, void *stream);

/* ---- timing hooks (HIP events on the sort's stream) ---- */
int labsort_timing_enable(int on);                /* clears accumulated times */
/* After the stream has been synchronised: total ms and launch count of a
 * kernel class (LABSORT_K_*) recorded since labsort_timing_enable(1). */
int labsort_timing_read(int kernel_class, double *total_ms, long long *launches);

/* ---- the north_star's entry name (the reference never defined it) ---- */
void sort(int *in, int n);

#ifdef __cplusplus
}
#endif
#endif /* LABSORT_H */
