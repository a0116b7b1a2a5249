/*! @file dist.h
 *  @brief Multi-GPU layer of the C library: one process drives every local
 *  MI355X ("single-process, multi-device"), RCCL over xGMI for collectives.
 *
 *  The reference has no parallelism beyond SIMD lanes; this header adds the
 *  parallel forms of its operations:
 *    - D2 data parallel:     vs_dist_conv1d_batch (batch sharded over ranks);
 *    - D3 tensor parallel:   vs_dist_sgemm_rowsplit (A rows sharded, B
 *                            broadcast, C rows downloaded per rank) and
 *                            vs_dist_sgemm_rowsplit_device (C all-gathered
 *                            in place on every GPU, per-matrix pipelined);
 *    - D4 context parallel:  vs_dist_conv1d_long / vs_dist_swt_long (long
 *                            signal split into contiguous chunks, halos
 *                            exchanged with neighbour send/recv);
 *    - D5 communicator:      vs_dist_create (ncclCommInitAll over distinct
 *                            devices, or the in-process LOCAL backend that
 *                            maps ranks onto any set of devices -- several
 *                            ranks may share one GPU -- and implements the
 *                            same collectives with stream-ordered copies).
 *  Every rank owns a non-blocking HIP stream on its device; collectives and
 *  sharded entry points are enqueued on those streams and the host-pointer
 *  entry points return after vs_dist_synchronize(), which polls RCCL's
 *  asynchronous error state and aborts the communicator after the timeout.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_DIST_H_
#define VELES_SIMD_DIST_H_

#include <stddef.h>
#include <stdint.h>

#include <simd/common.h>
#include <simd/gpu.h>

SIMD_API_BEGIN

typedef struct vs_dist_context *vs_dist_t;

typedef enum {
  VS_DIST_AUTO = 0,   ///< RCCL when every rank has its own device, else LOCAL
  VS_DIST_RCCL = 1,   ///< ncclCommInitAll over distinct devices
  VS_DIST_LOCAL = 2   ///< stream-ordered copies; ranks may share a device
} vs_dist_backend;

/// Creates a communicator of `nranks` ranks.  `devices` (may be NULL: rank r
/// -> device r mod device_count) lists the device of each rank.
vs_status vs_dist_create(int nranks, const int *devices, int backend,
                         vs_dist_t *out);
vs_status vs_dist_destroy(vs_dist_t ctx);
int vs_dist_size(vs_dist_t ctx);
int vs_dist_backend_of(vs_dist_t ctx);
int vs_dist_device(vs_dist_t ctx, int rank);
vs_stream_t vs_dist_stream(vs_dist_t ctx, int rank);
/// Watchdog for vs_dist_synchronize (milliseconds, 0 = wait forever;
/// default 300000 or VELES_DIST_TIMEOUT_MS).
vs_status vs_dist_set_timeout(vs_dist_t ctx, int ms);
/// Waits for every rank stream.  Polls ncclCommGetAsyncError while waiting;
/// on an RCCL error or timeout aborts the communicator and returns
/// VS_ERR_COMM / VS_ERR_TIMEOUT (the context is then unusable).
vs_status vs_dist_synchronize(vs_dist_t ctx);

/// Contiguous shard of n items for `rank`: the first n % nranks ranks get
/// one extra item.  Pure host arithmetic.
void vs_dist_shard(size_t n, int nranks, int rank, size_t *begin,
                   size_t *count);

/* ------------------------------------------- collectives (device buffers)
 * bufs[r] / send[r] / recv[r] are device pointers on rank r's device. */
vs_status vs_dist_broadcast(vs_dist_t ctx, void *const *bufs, size_t bytes,
                            int root);
/// recv[r] = concat over q of send[q] (bytes_per_rank each).
vs_status vs_dist_all_gather(vs_dist_t ctx, const void *const *send,
                             void *const *recv, size_t bytes_per_rank);
/// In-place float sum over ranks.
vs_status vs_dist_all_reduce_sum(vs_dist_t ctx, float *const *bufs, size_t n);
/// Neighbour halo exchange.  direction +1: halo[r] = last halo_len floats of
/// src[r-1] (rank 0 gets the tail of the last rank if periodic, else
/// zeros); direction -1: halo[r] = first halo_len floats of src[r+1] (the
/// last rank gets the head of rank 0 if periodic, else zeros).
/// src_len[r] >= halo_len is required.
vs_status vs_dist_halo_exchange(vs_dist_t ctx, const float *const *src,
                                const size_t *src_len, float *const *halo,
                                size_t halo_len, int direction, int periodic);

/* ------------------------------ sharded entry points (host pointers in/out) */
/// C[b] = A[b] @ B[b] for b < batch (row-major host arrays, A [batch][m][k],
/// B [batch][k][n], C [batch][m][n]): rows of A split over ranks (each rank
/// uploads and holds only its rows), B uploaded once to rank 0 and
/// broadcast over xGMI, and each rank downloads its own C rows straight into
/// the caller's C on a second stream, overlapping the next matrix's GEMM.
/// No rank ever holds the whole C, so nothing is gathered.
vs_status vs_dist_sgemm_rowsplit(vs_dist_t ctx, int m, int n, int k,
                                 const float *A, const float *B, float *C,
                                 int batch);
/// Device-resident form for consumers that need the whole product on every
/// GPU (benchmark config 5): A[r] is rank r's rows ([batch][rows_r][k] on
/// its device, rows_r from vs_dist_shard(m, size, r)), B[r] the full
/// [batch][k][n] on rank r, C[r] a [batch][m][n] buffer on rank r.  Each
/// rank computes its rows in place in its C[r]; the row blocks of matrix b
/// are all-gathered in place (RCCL: one group of broadcasts, one root per
/// rank) on the side streams while matrix b + 1 is multiplied.  Returns
/// with every rank's main stream ordered after the gather.
vs_status vs_dist_sgemm_rowsplit_device(vs_dist_t ctx, int m, int n, int k,
                                        const float *const *A, const float *const *B,
                                        float *const *C, int batch);
/// Data-parallel batched convolution / correlation: rows of x [batch][x_len]
/// sharded over ranks, one shared filter h, y [batch][x_len + h_len - 1].
vs_status vs_dist_conv1d_batch(vs_dist_t ctx, int correlate, const float *x,
                               int x_len, const float *h, int h_len, float *y,
                               int batch);
/// Data-parallel batches, rows (matrices) sharded over ranks with
/// vs_dist_shard, no communication.  Stationary wavelet transform of
/// x [batch][len]: hi [batch][levels][len], lo [batch][len] (the layout of
/// vs_swt_multilevel; reference src/wavelet.c:1907-1940, one signal and one
/// level per call).
vs_status vs_dist_swt_batch(vs_dist_t ctx, int type, int order, int levels, int ext,
                            const float *x, int len, int batch, float *hi, float *lo);
/// Device-resident form: x[r] / hi[r] / lo[r] are rank r's rows on its
/// device, batch[r] its row count; enqueued on the ranks' main streams
/// (vs_dist_synchronize or vs_dist_stream to order after it).
vs_status vs_dist_swt_batch_device(vs_dist_t ctx, int type, int order, int levels, int ext,
                                   const float *const *x, int len, const int *batch,
                                   float *const *hi, float *const *lo);
/// Decimated pyramid of x [batch][len]: out [batch][len] rows
/// [hi_1 | hi_2 | ... | hi_L | lo_L] (vs_dwt_multilevel).
vs_status vs_dist_dwt_batch(vs_dist_t ctx, int type, int order, int levels, int ext,
                            const float *x, int len, int batch, float *out);
/// C[b] = op(A[b]) op(B[b]) for b < batch, the matrices sharded over ranks
/// (A [batch][m][k] or [batch][k][m] when trans_a, B likewise, C [batch][m][n]).
vs_status vs_dist_sgemm_batch(vs_dist_t ctx, int trans_a, int trans_b, int m, int n, int k,
                              const float *A, const float *B, float *C, int batch);
/// Context-parallel convolution / correlation of one long signal: x split
/// into contiguous chunks (each >= h_len - 1), rank r receives the last
/// h_len - 1 samples of rank r-1 as history and writes its disjoint slice of
/// y (length x_len + h_len - 1; the last rank also the h_len - 1 tail).
vs_status vs_dist_conv1d_long(vs_dist_t ctx, int correlate, const float *x,
                              size_t x_len, const float *h, int h_len,
                              float *y);
/// Context-parallel stationary DWT of one long signal, levels 1..levels
/// (level l fed by level l-1's lo): hi [levels][len], lo [len] (last
/// level).  Per level, rank r < last receives the first
/// (order - 1) 2^(l-1) samples of rank r+1; the last rank extends
/// periodically from rank 0 or locally (mirror / constant / zero).
vs_status vs_dist_swt_long(vs_dist_t ctx, int type, int order, int levels,
                           int ext, const float *x, size_t len, float *hi,
                           float *lo);

SIMD_API_END

#endif  // VELES_SIMD_DIST_H_
