/* vv_dsp_dist.h -- multi-GPU layout of the spectral path (SURVEY.md 8e,
 * BASELINE config 5: "256 ch x 10 min sharded across 8 x MI355X, RCCL gather
 * over xGMI") in plain C over RCCL.
 *
 * The path shards with NO data-path exchange: channels (STFT, FIR) and
 * transforms (batched FFT) are independent, so rank r of `world` computes the
 * contiguous block vv_dsp_shard_range(total, world, r) on its own GPU.  The one
 * collective is the gather of the result rows to a root rank, done as
 * point-to-point ncclSend / ncclRecv slabs (xGMI is point-to-point: the root's
 * 7 links each carry one peer's slab), optionally with half-spectrum rows.
 *
 * A context holds the ranks THIS process drives ("local slots"): all of them
 * (vv_dsp_dist_init_all, one process for the node, ncclCommInitAll), one
 * (vv_dsp_dist_from_comm, one process per GPU with the caller's communicator),
 * or a loopback set of ranks on one device whose transfers are device copies
 * (vv_dsp_dist_init_loopback: the layout and the slab logic at world > 1 on a
 * single GPU).  Every per-rank array argument below has one element per local
 * slot, on that slot's device.  librccl.so.1 is loaded on first use
 * (UNSUPPORTED if it is missing); nothing here changes the reference's API. */
#ifndef VV_DSP_DIST_H
#define VV_DSP_DIST_H
#include "vv_dsp/vv_dsp_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vv_dsp_dist vv_dsp_dist;

#define VV_DSP_DIST_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES */

/* ndev ranks in this process, rank i on devices[i] (ncclCommInitAll). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_init_all(int ndev, const int* devices, vv_dsp_dist** out);
/* One process per GPU: rank 0 makes an id (ncclGetUniqueId) and hands its
 * VV_DSP_DIST_ID_BYTES bytes to every rank by any means (e.g. a broadcast of the
 * job's launcher); each rank then joins with vv_dsp_dist_init_rank
 * (ncclCommInitRank, collective over the `world` ranks) with its rank and the
 * device it runs on.  The communicator is the context's own: vv_dsp_dist_destroy
 * destroys it. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_unique_id(unsigned char id[VV_DSP_DIST_ID_BYTES]);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_init_rank(int world, int rank, const unsigned char id[VV_DSP_DIST_ID_BYTES],
                                                     int device, vv_dsp_dist** out);
/* One rank of a communicator the caller made (an ncclComm_t passed as void*,
 * e.g. ncclCommInitRank in a one-process-per-GPU job); rank, world size and
 * device are read from it, and vv_dsp_dist_destroy leaves it alone. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_from_comm(void* nccl_comm, vv_dsp_dist** out);
/* `world` ranks on ONE device in this process, their transfers done as device
 * copies instead of RCCL messages; every operation runs on streams[root]. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_init_loopback(int world, int device, vv_dsp_dist** out);
vv_dsp_status vv_dsp_dist_destroy(vv_dsp_dist* d);
/* ranks this process drives = the length of every per-rank array below */
int vv_dsp_dist_local_ranks(const vv_dsp_dist* d);
/* local slot s: its rank, the world size and its device */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_rank_info(const vv_dsp_dist* d, int slot, int* rank, int* world,
                                                     int* device);
/* the rank count RCCL reports for slot s's communicator (ncclCommCount; the
 * world size for a loopback context) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_comm_count(const vv_dsp_dist* d, int slot, int* count);

/* Streams: every per-rank `streams` array has one hipStream_t per local slot,
 * each on that slot's device (OUT_OF_RANGE otherwise; NULL = the device's null
 * stream).  Work for slot s is enqueued on streams[s] with its device current. */

/* Config 5: each local rank's share of a [total_ch][n] multi-channel STFT --
 * the channels vv_dsp_shard_range(total_ch, world, rank) gives it, d_signal[s]
 * pointing at that shard's first channel (ch_stride floats apart) -- into
 * d_rows[s] = [count][frames][row], out_kind 0 magnitude (row = fft_size
 * floats), 1 complex (fft_size vv_dsp_cpx), 2 power (fft_size/2+1 floats).
 * The rows are bit-identical to one vv_dsp_stft_spectrogram_device call over
 * all channels (frames never span channels). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_stft(vv_dsp_dist* d, vv_dsp_stft* h, const vv_dsp_real* const* d_signal,
                                                size_t n, size_t total_ch, size_t ch_stride, int out_kind,
                                                void* const* d_rows, void* const* streams, size_t* out_frames);
/* The gather: every rank's items d_local[s] = [count_r][rows_per_item][row_floats]
 * (count_r from vv_dsp_shard_range(total_items, world, r): channels of a
 * spectrogram, rows_per_item = its frames) into d_root_out =
 * [total_items][rows_per_item][row_floats] on rank `root` (ignored on other
 * ranks), in rank = item order, in slabs of at most 256 MiB per rank (a slab
 * may end inside an item; every rank derives the same slab bounds).  The
 * root's own rows may already sit at their place in d_root_out (no copy then).
 * half != 0: the rows MUST be mirror-symmetric rows of fft_size = row_floats
 * bins (row[k] == row[fft_size - k]: magnitude rows of real frames -- never
 * the fft_size/2+1-wide power rows, which are gathered with half = 0); each
 * rank sends bins 0..fft_size/2 only and the root expands them
 * (vv_dsp_spectrogram_pack/unpack_half_device): the same rows for half the
 * xGMI bytes.  Stream-ordered: returns once everything is enqueued; the
 * sources must be complete in stream order on streams[s].  half != 0 with an
 * odd row_floats is INVALID_SIZE.  Loopback contexts run every copy on
 * streams[root], after a device-side wait for each streams[s]; afterwards each
 * streams[s] waits (device side) for streams[root], so work the caller enqueues
 * on streams[s] after the call (e.g. the next step's rows into d_local[s]) runs
 * after the gather has read d_local[s] -- as on the RCCL path, whose sends run on
 * streams[s]. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_gather_rows(vv_dsp_dist* d, const vv_dsp_real* const* d_local,
                                                       size_t total_items, size_t rows_per_item, size_t row_floats,
                                                       int half, vv_dsp_real* d_root_out, int root,
                                                       void* const* streams);
/* Config 2: each local rank transforms its batch shard -- transforms
 * vv_dsp_shard_range(total_batch, world, rank) of a [total_batch][n] job, d_in[s]
 * / d_out[s] pointing at the shard's first transform (layout as
 * vv_dsp_fft_execute_device). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_fft(vv_dsp_dist* d, size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir,
                                               size_t total_batch, const void* const* d_in, void* const* d_out,
                                               void* const* streams);
/* Config 4: each local rank filters its channel shard of a [total_ch][n] job
 * (overlap-save, vv_dsp_fir_apply_fft_device) with plans[s], a plan created
 * while slot s's device was current (its filter spectrum lives there). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dist_fir_apply_fft(vv_dsp_dist* d, vv_dsp_fir_plan* const* plans, size_t n,
                                                         size_t total_ch, const vv_dsp_real* const* d_x,
                                                         size_t x_stride, vv_dsp_real* const* d_y, size_t y_stride,
                                                         void* const* streams);

#ifdef __cplusplus
}
#endif
#endif
