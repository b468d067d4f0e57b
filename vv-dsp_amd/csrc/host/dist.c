/* dist.c -- multi-GPU layout of the spectral path in plain C over RCCL
 * (include/vv_dsp/vv_dsp_dist.h; SURVEY.md 8e, BASELINE config 5).
 *
 * Shards: rank r of `world` owns the contiguous block vv_dsp_shard_range(total,
 * world, r) of channels (STFT, FIR) or transforms (FFT) and computes it on its
 * own GPU with the single-GPU kernels -- no exchange in the data path.
 *
 * Gather (config 5's "RCCL gather over xGMI"): slab k of every rank's rows goes
 * to the root as one ncclSend / ncclRecv pair per peer inside one
 * ncclGroupStart/End.  RCCL's ncclGather needs equal counts per rank; the
 * pairs take the channel_shard layout's uneven sizes as they are and land each
 * full row straight at its final offset of the root's output (no padding, no
 * staging).  With half rows each rank packs bins 0..nfft/2 of its slab first
 * and the root receives into one staging slab per peer and expands them.
 * Slabs are at most 256 MiB per rank: messages stay far below 2^31 elements
 * (a config-5 shard is 3.7e9 floats) and staging stays small.
 *
 * RCCL is dlopen'ed on first use (librccl.so.1, the soname torch's copy shares
 * when it is already loaded), so the library itself does not depend on it. */
#include "vv_dsp/vv_dsp_dist.h"
#include "vv_dsp_hip.h"

#include <dlfcn.h>
#include <pthread.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define DIST_MAX_SLOTS 64
#ifndef DIST_SLAB_BYTES /* a test-only build (tests/distsim) compiles a small slab in */
#define DIST_SLAB_BYTES ((size_t)256 << 20)
#endif

/* ---- RCCL entry points, resolved at run time ---- */
static struct {
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*);
    ncclResult_t (*unique_id)(ncclUniqueId*);
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*destroy)(ncclComm_t);
    ncclResult_t (*group_start)(void);
    ncclResult_t (*group_end)(void);
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    const char* (*err)(ncclResult_t);
    ncclResult_t (*count)(const ncclComm_t, int*);
    ncclResult_t (*user_rank)(const ncclComm_t, int*);
    ncclResult_t (*cu_device)(const ncclComm_t, int*);
    int ok;
} R;
static pthread_once_t r_once = PTHREAD_ONCE_INIT;

static void rccl_load(void) {
    void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!so) return;
#define SYM(field, name)                                   \
    do {                                                   \
        *(void**)(&R.field) = dlsym(so, name);             \
        if (!R.field) return;                              \
    } while (0)
    SYM(init_all, "ncclCommInitAll");
    SYM(unique_id, "ncclGetUniqueId");
    SYM(init_rank, "ncclCommInitRank");
    SYM(destroy, "ncclCommDestroy");
    SYM(group_start, "ncclGroupStart");
    SYM(group_end, "ncclGroupEnd");
    SYM(send, "ncclSend");
    SYM(recv, "ncclRecv");
    SYM(err, "ncclGetErrorString");
    SYM(count, "ncclCommCount");
    SYM(user_rank, "ncclCommUserRank");
    SYM(cu_device, "ncclCommCuDevice");
#undef SYM
    R.ok = 1;
}

static int rccl_ready(void) {
    pthread_once(&r_once, rccl_load);
    if (!R.ok) vvhip_set_error("librccl.so.1 (RCCL) could not be loaded");
    return R.ok;
}

static vv_dsp_status nccl_fail(const char* what, ncclResult_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, R.err ? R.err(e) : "rccl error");
    vvhip_set_error(buf);
    return VV_DSP_ERROR_INTERNAL;
}

struct vv_dsp_dist {
    int nslots, world;
    int rank[DIST_MAX_SLOTS], dev[DIST_MAX_SLOTS];
    ncclComm_t comm[DIST_MAX_SLOTS];
    int own_comms;   /* created here: destroyed by vv_dsp_dist_destroy */
    int loopback;    /* all ranks in this process on one device, transfers are copies */
    int one_process; /* every rank of the world is a slot of this context (init_all,
                        loopback): only then may the slab size follow a per-process knob */
};

static vv_dsp_dist* dist_new(void) { return (vv_dsp_dist*)calloc(1, sizeof(vv_dsp_dist)); }

vv_dsp_status vv_dsp_dist_init_all(int ndev, const int* devices, vv_dsp_dist** out) {
    if (!out || !devices) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (ndev < 1 || ndev > DIST_MAX_SLOTS) return VV_DSP_ERROR_INVALID_SIZE;
    const int nd = vvhip_available();
    if (nd <= 0) return VV_DSP_ERROR_UNSUPPORTED;
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= nd) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (!rccl_ready()) return VV_DSP_ERROR_UNSUPPORTED;
    vv_dsp_dist* d = dist_new();
    if (!d) return VV_DSP_ERROR_INTERNAL;
    ncclResult_t e = R.init_all(d->comm, ndev, devices);
    if (e != ncclSuccess) {
        free(d);
        return nccl_fail("ncclCommInitAll", e);
    }
    d->nslots = d->world = ndev;
    d->own_comms = 1;
    d->one_process = 1;
    for (int i = 0; i < ndev; ++i) {
        d->rank[i] = i;
        d->dev[i] = devices[i];
    }
    *out = d;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_from_comm(void* nccl_comm, vv_dsp_dist** out) {
    if (!out || !nccl_comm) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (vvhip_available() <= 0) return VV_DSP_ERROR_UNSUPPORTED;
    if (!rccl_ready()) return VV_DSP_ERROR_UNSUPPORTED;
    vv_dsp_dist* d = dist_new();
    if (!d) return VV_DSP_ERROR_INTERNAL;
    ncclComm_t c = (ncclComm_t)nccl_comm;
    ncclResult_t e = R.count(c, &d->world);
    if (e == ncclSuccess) e = R.user_rank(c, &d->rank[0]);
    if (e == ncclSuccess) e = R.cu_device(c, &d->dev[0]);
    if (e != ncclSuccess) {
        free(d);
        return nccl_fail("communicator query", e);
    }
    d->nslots = 1;
    d->comm[0] = c;
    *out = d;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_unique_id(unsigned char id[VV_DSP_DIST_ID_BYTES]) {
    if (!id) return VV_DSP_ERROR_NULL_POINTER;
    if (!rccl_ready()) return VV_DSP_ERROR_UNSUPPORTED;
    ncclUniqueId u;
    const ncclResult_t e = R.unique_id(&u);
    if (e != ncclSuccess) return nccl_fail("ncclGetUniqueId", e);
    memcpy(id, u.internal, VV_DSP_DIST_ID_BYTES);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_init_rank(int world, int rank, const unsigned char id[VV_DSP_DIST_ID_BYTES], int device,
                                    vv_dsp_dist** out) {
    if (!out || !id) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (world < 1) return VV_DSP_ERROR_INVALID_SIZE;
    if (rank < 0 || rank >= world) return VV_DSP_ERROR_OUT_OF_RANGE;
    const int nd = vvhip_available();
    if (nd <= 0) return VV_DSP_ERROR_UNSUPPORTED;
    if (device < 0 || device >= nd) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (!rccl_ready()) return VV_DSP_ERROR_UNSUPPORTED;
    vv_dsp_dist* d = dist_new();
    if (!d) return VV_DSP_ERROR_INTERNAL;
    ncclUniqueId u;
    memcpy(u.internal, id, VV_DSP_DIST_ID_BYTES);
    /* the communicator binds to the current device */
    int prev = 0;
    if (vvhip_get_device(&prev) != 0 || vvhip_set_device(device) != 0) {
        free(d);
        return VV_DSP_ERROR_INTERNAL;
    }
    const ncclResult_t e = R.init_rank(&d->comm[0], world, u, rank);
    (void)vvhip_set_device(prev);
    if (e != ncclSuccess) {
        free(d);
        return nccl_fail("ncclCommInitRank", e);
    }
    d->nslots = 1;
    d->world = world;
    d->rank[0] = rank;
    d->dev[0] = device;
    d->own_comms = 1;
    *out = d;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_init_loopback(int world, int device, vv_dsp_dist** out) {
    if (!out) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (world < 1 || world > DIST_MAX_SLOTS) return VV_DSP_ERROR_INVALID_SIZE;
    const int nd = vvhip_available();
    if (nd <= 0) return VV_DSP_ERROR_UNSUPPORTED;
    if (device < 0 || device >= nd) return VV_DSP_ERROR_OUT_OF_RANGE;
    vv_dsp_dist* d = dist_new();
    if (!d) return VV_DSP_ERROR_INTERNAL;
    d->nslots = d->world = world;
    d->loopback = 1;
    d->one_process = 1;
    for (int i = 0; i < world; ++i) {
        d->rank[i] = i;
        d->dev[i] = device;
    }
    *out = d;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_destroy(vv_dsp_dist* d) {
    if (!d) return VV_DSP_ERROR_NULL_POINTER;
    vv_dsp_status st = VV_DSP_OK;
    if (d->own_comms)
        for (int i = 0; i < d->nslots; ++i)
            if (R.destroy(d->comm[i]) != ncclSuccess) st = VV_DSP_ERROR_INTERNAL;
    free(d);
    return st;
}

int vv_dsp_dist_local_ranks(const vv_dsp_dist* d) { return d ? d->nslots : 0; }

vv_dsp_status vv_dsp_dist_rank_info(const vv_dsp_dist* d, int slot, int* rank, int* world, int* device) {
    if (!d) return VV_DSP_ERROR_NULL_POINTER;
    if (slot < 0 || slot >= d->nslots) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (rank) *rank = d->rank[slot];
    if (world) *world = d->world;
    if (device) *device = d->dev[slot];
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_comm_count(const vv_dsp_dist* d, int slot, int* count) {
    if (!d || !count) return VV_DSP_ERROR_NULL_POINTER;
    if (slot < 0 || slot >= d->nslots) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (d->loopback) {
        *count = d->world;
        return VV_DSP_OK;
    }
    const ncclResult_t e = R.count(d->comm[slot], count);
    return e == ncclSuccess ? VV_DSP_OK : nccl_fail("ncclCommCount", e);
}

/* ---- layout helpers (vv_dsp_amd.h) ---- */
vv_dsp_status vv_dsp_shard_range(size_t total, size_t world, size_t rank, size_t* first, size_t* count) {
    if (!first || !count) return VV_DSP_ERROR_NULL_POINTER;
    if (world == 0 || rank >= world) return VV_DSP_ERROR_OUT_OF_RANGE;
    const size_t base = total / world, rem = total % world;
    *first = rank * base + (rank < rem ? rank : rem);
    *count = base + (rank < rem ? 1 : 0);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_spectrogram_pack_half_device(const vv_dsp_real* d_rows, size_t rows, size_t fft_size,
                                                  vv_dsp_real* d_half, void* stream) {
    if (!d_rows || !d_half) return VV_DSP_ERROR_NULL_POINTER;
    if (fft_size == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_rows_half_device(d_rows, d_half, rows, fft_size, 0, stream);
}

vv_dsp_status vv_dsp_spectrogram_unpack_half_device(const vv_dsp_real* d_half, size_t rows, size_t fft_size,
                                                    vv_dsp_real* d_rows, void* stream) {
    if (!d_half || !d_rows) return VV_DSP_ERROR_NULL_POINTER;
    if (fft_size == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_rows_half_device(d_half, d_rows, rows, fft_size, 1, stream);
}

/* ---- helpers ---- */
static size_t shard_first(size_t total, int world, int r) {
    size_t first = 0, count = 0;
    return vv_dsp_shard_range(total, (size_t)world, (size_t)r, &first, &count) == VV_DSP_OK ? first : 0;
}
static size_t shard_count(size_t total, int world, int r) {
    size_t first = 0, count = 0;
    return vv_dsp_shard_range(total, (size_t)world, (size_t)r, &first, &count) == VV_DSP_OK ? count : 0;
}

/* runs with slot s's device current; restores the caller's device */
typedef struct {
    int prev, ok;
} dev_scope;
static vv_dsp_status dev_enter(dev_scope* g, int dev) {
    g->ok = vvhip_get_device(&g->prev) == 0;
    if (!g->ok) return VV_DSP_ERROR_INTERNAL;
    return vvhip_set_device(dev) == 0 ? VV_DSP_OK : VV_DSP_ERROR_INTERNAL;
}
static vv_dsp_status dev_leave(const dev_scope* g, vv_dsp_status st) {
    if (g->ok && vvhip_set_device(g->prev) != 0 && st == VV_DSP_OK) st = VV_DSP_ERROR_INTERNAL;
    return st;
}

static int slot_of_rank(const vv_dsp_dist* d, int r) {
    for (int s = 0; s < d->nslots; ++s)
        if (d->rank[s] == r) return s;
    return -1;
}

/* every non-null stream must belong to its slot's device (work for slot s is
 * enqueued with d->dev[s] current; a null stream is that device's null stream) */
static vv_dsp_status check_streams(const vv_dsp_dist* d, void* const* streams) {
    for (int s = 0; s < d->nslots; ++s) {
        if (!streams[s]) continue;
        int dev = -1;
        if (vvhip_stream_device(streams[s], &dev) != 0) return VV_DSP_ERROR_INTERNAL;
        if (dev != d->dev[s]) {
            char buf[160];
            snprintf(buf, sizeof buf, "dist: the stream of slot %d is on device %d, the slot's rank runs on device %d", s,
                     dev, d->dev[s]);
            vvhip_set_error(buf);
            return VV_DSP_ERROR_OUT_OF_RANGE;
        }
    }
    return VV_DSP_OK;
}

static vv_dsp_status check_arrays(const vv_dsp_dist* d, const void* a, const void* b, void* const* streams) {
    if (!d || !a || !b || !streams) return VV_DSP_ERROR_NULL_POINTER;
    return check_streams(d, streams);
}

/* ---- shards ---- */
vv_dsp_status vv_dsp_dist_stft(vv_dsp_dist* d, vv_dsp_stft* h, const vv_dsp_real* const* d_signal, size_t n,
                               size_t total_ch, size_t ch_stride, int out_kind, void* const* d_rows,
                               void* const* streams, size_t* out_frames) {
    vv_dsp_status st = check_arrays(d, d_signal, d_rows, streams);
    if (st != VV_DSP_OK) return st;
    if (!h) return VV_DSP_ERROR_NULL_POINTER;
    if (out_kind < 0 || out_kind > 2) return VV_DSP_ERROR_OUT_OF_RANGE;
    size_t nfft = 0, hop = 0;
    st = vv_dsp_stft_get_sizes(h, &nfft, &hop);
    if (st != VV_DSP_OK) return st;
    const size_t frames = vvhip_stft_num_frames(n, nfft, hop);
    const size_t row = out_kind == 2 ? nfft / 2 + 1 : nfft;
    if (out_frames) *out_frames = frames;
    for (int s = 0; s < d->nslots; ++s) {
        const size_t cnt = shard_count(total_ch, d->world, d->rank[s]);
        if (cnt == 0) continue;
        if (!d_signal[s] || !d_rows[s]) return VV_DSP_ERROR_NULL_POINTER;
        size_t fr = 0;
        st = vv_dsp_stft_channel_shard_device(h, d->dev[s], d_signal[s], n, cnt, ch_stride, out_kind, d_rows[s],
                                              frames * row, streams[s], &fr);
        if (st != VV_DSP_OK) return st;
    }
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_fft(vv_dsp_dist* d, size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir, size_t total_batch,
                              const void* const* d_in, void* const* d_out, void* const* streams) {
    vv_dsp_status st = check_arrays(d, d_in, d_out, streams);
    if (st != VV_DSP_OK) return st;
    for (int s = 0; s < d->nslots; ++s) {
        const size_t cnt = shard_count(total_batch, d->world, d->rank[s]);
        if (cnt == 0) continue;
        if (!d_in[s] || !d_out[s]) return VV_DSP_ERROR_NULL_POINTER;
        dev_scope g;
        st = dev_enter(&g, d->dev[s]);
        vv_dsp_fft_plan* p = NULL;
        if (st == VV_DSP_OK) st = vv_dsp_fft_make_plan_many(n, type, dir, cnt, &p);
        if (st == VV_DSP_OK) st = vv_dsp_fft_execute_device(p, d_in[s], d_out[s], streams[s]);
        if (p) (void)vv_dsp_fft_destroy(p);   /* nothing enqueued reads the plan */
        st = dev_leave(&g, st);
        if (st != VV_DSP_OK) return st;
    }
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dist_fir_apply_fft(vv_dsp_dist* d, vv_dsp_fir_plan* const* plans, size_t n, size_t total_ch,
                                        const vv_dsp_real* const* d_x, size_t x_stride, vv_dsp_real* const* d_y,
                                        size_t y_stride, void* const* streams) {
    vv_dsp_status st = check_arrays(d, d_x, d_y, streams);
    if (st != VV_DSP_OK) return st;
    if (!plans) return VV_DSP_ERROR_NULL_POINTER;
    for (int s = 0; s < d->nslots; ++s) {
        const size_t cnt = shard_count(total_ch, d->world, d->rank[s]);
        if (cnt == 0) continue;
        if (!plans[s] || !d_x[s] || !d_y[s]) return VV_DSP_ERROR_NULL_POINTER;
        dev_scope g;
        st = dev_enter(&g, d->dev[s]);
        if (st == VV_DSP_OK) st = vv_dsp_fir_apply_fft_device(plans[s], d_x[s], d_y[s], n, cnt, x_stride, y_stride, streams[s]);
        st = dev_leave(&g, st);
        if (st != VV_DSP_OK) return st;
    }
    return VV_DSP_OK;
}

/* ---- the gather ---- */
/* rank r's rows: items vv_dsp_shard_range(total_items, world, r), rows_per_item each */
static size_t rows_first(size_t total_items, size_t rpi, int world, int r) { return shard_first(total_items, world, r) * rpi; }
static size_t rows_count(size_t total_items, size_t rpi, int world, int r) { return shard_count(total_items, world, r) * rpi; }

vv_dsp_status vv_dsp_dist_gather_rows(vv_dsp_dist* d, const vv_dsp_real* const* d_local, size_t total_items,
                                      size_t rows_per_item, size_t row_floats, int half, vv_dsp_real* d_root_out,
                                      int root, void* const* streams) {
    if (!d || !d_local || !streams) return VV_DSP_ERROR_NULL_POINTER;
    if (row_floats == 0 || rows_per_item == 0) return VV_DSP_ERROR_INVALID_SIZE;
    /* half rows: bins 0..row_floats/2 of an even-length mirror-symmetric row
     * (an odd width is a power row or some other non-mirror row: refused) */
    if (half && (row_floats < 2 || row_floats % 2 != 0)) {
        vvhip_set_error("dist gather: half rows need an even row_floats (mirror-symmetric fft_size-bin rows)");
        return VV_DSP_ERROR_INVALID_SIZE;
    }
    if (root < 0 || root >= d->world) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (!d->loopback && !rccl_ready()) return VV_DSP_ERROR_UNSUPPORTED;
    vv_dsp_status st = check_streams(d, streams);
    if (st != VV_DSP_OK) return st;
    const int world = d->world, rs = slot_of_rank(d, root);
    if (rs >= 0 && !d_root_out) return VV_DSP_ERROR_NULL_POINTER;
    for (int s = 0; s < d->nslots; ++s)
        if (!d_local[s] && rows_count(total_items, rows_per_item, world, d->rank[s]) > 0) return VV_DSP_ERROR_NULL_POINTER;
    const size_t w = half ? row_floats / 2 + 1 : row_floats;   /* floats sent per row */
    size_t cmax = 0;
    for (int r = 0; r < world; ++r) {
        const size_t c = rows_count(total_items, rows_per_item, world, r);
        if (c > cmax) cmax = c;
    }
    if (cmax == 0) return VV_DSP_OK;
    /* knob (tests): a smaller slab -- only where one process drives every rank,
     * since the sender and the root each derive the slab bounds */
    const long long kb = d->one_process ? vvhip_debug_get("DIST_SLAB_KB") : -1;
    size_t slab = (kb > 0 ? (size_t)kb << 10 : DIST_SLAB_BYTES) / (sizeof(float) * w);
    if (slab < 1) slab = 1;
    if (slab > cmax) slab = cmax;

    /* the root's own rows: one device copy to their place (no-op in place) */
    if (rs >= 0) {
        const size_t c = rows_count(total_items, rows_per_item, world, root);
        dev_scope g;
        st = dev_enter(&g, d->dev[rs]);
        if (st == VV_DSP_OK && c)
            st = vvhip_memcpy_d2d_async(d_root_out + rows_first(total_items, rows_per_item, world, root) * row_floats, d_local[rs],
                                        sizeof(float) * c * row_floats, streams[rs]) == 0
                     ? VV_DSP_OK
                     : VV_DSP_ERROR_INTERNAL;
        st = dev_leave(&g, st);
        if (st != VV_DSP_OK) return st;
    }
    if (world == 1) return VV_DSP_OK;
    void* const rstream = rs >= 0 ? streams[rs] : NULL;
    /* loopback: every pack, copy and unpack runs on the root's stream, so it
     * first waits for each slot's stream, where that slot's rows were written */
    if (d->loopback)
        for (int s = 0; s < d->nslots && st == VV_DSP_OK; ++s)
            if (s != rs && vvhip_stream_wait(rstream, streams[s]) != 0) st = VV_DSP_ERROR_INTERNAL;
    if (st != VV_DSP_OK) return st;

    /* scratch: a packed slab per sending slot (half rows); on the root one
     * staging slab per peer (half rows; full rows land in place) */
    float* pack[DIST_MAX_SLOTS] = {0};
    float* stage = NULL;
    if (half) {
        for (int s = 0; s < d->nslots && st == VV_DSP_OK; ++s) {
            if (d->rank[s] == root || rows_count(total_items, rows_per_item, world, d->rank[s]) == 0) continue;
            dev_scope g;
            st = dev_enter(&g, d->dev[s]);
            void* sp = d->loopback ? rstream : streams[s];
            if (st == VV_DSP_OK && vvhip_malloc_async((void**)&pack[s], sizeof(float) * slab * w, sp) != 0)
                st = VV_DSP_ERROR_INTERNAL;
            st = dev_leave(&g, st);
        }
        if (st == VV_DSP_OK && rs >= 0) {
            dev_scope g;
            st = dev_enter(&g, d->dev[rs]);
            if (st == VV_DSP_OK && vvhip_malloc_async((void**)&stage, sizeof(float) * (size_t)world * slab * w, rstream) != 0)
                st = VV_DSP_ERROR_INTERNAL;
            st = dev_leave(&g, st);
        }
    }

    for (size_t i0 = 0; i0 < cmax && st == VV_DSP_OK; i0 += slab) {
        /* 1. senders pack their slab (half rows) */
        if (half)
            for (int s = 0; s < d->nslots && st == VV_DSP_OK; ++s) {
                const int r = d->rank[s];
                const size_t c = rows_count(total_items, rows_per_item, world, r);
                if (r == root || i0 >= c) continue;
                const size_t cnt = c - i0 < slab ? c - i0 : slab;
                dev_scope g;
                st = dev_enter(&g, d->dev[s]);
                if (st == VV_DSP_OK)
                    st = vv_dsp_spectrogram_pack_half_device(d_local[s] + i0 * row_floats, cnt, row_floats, pack[s],
                                                             d->loopback ? rstream : streams[s]);
                st = dev_leave(&g, st);
            }
        if (st != VV_DSP_OK) break;
        /* 2. the transfers of this slab: peer r's rows [i0, i0 + cnt) */
        if (d->loopback) {
            for (int r = 0; r < world && st == VV_DSP_OK; ++r) {
                const size_t c = rows_count(total_items, rows_per_item, world, r);
                if (r == root || i0 >= c) continue;
                const size_t cnt = c - i0 < slab ? c - i0 : slab;
                const int s = slot_of_rank(d, r);
                const float* src = half ? pack[s] : d_local[s] + i0 * row_floats;
                float* dst = half ? stage + (size_t)r * slab * w
                                  : d_root_out + (rows_first(total_items, rows_per_item, world, r) + i0) * row_floats;
                if (vvhip_memcpy_d2d_async(dst, src, sizeof(float) * cnt * w, rstream) != 0) st = VV_DSP_ERROR_INTERNAL;
            }
        } else {
            /* one group per slab: the root's receives from every peer and this
             * process's sends; on an error the group is still closed */
            ncclResult_t e = R.group_start();
            const char* what = "ncclGroupStart";
            for (int s = 0; s < d->nslots && e == ncclSuccess; ++s) {
                const int r = d->rank[s];
                if (r == root) {
                    for (int p = 0; p < world && e == ncclSuccess; ++p) {
                        const size_t c = rows_count(total_items, rows_per_item, world, p);
                        if (p == root || i0 >= c) continue;
                        const size_t cnt = c - i0 < slab ? c - i0 : slab;
                        float* dst = half ? stage + (size_t)p * slab * w
                                          : d_root_out + (rows_first(total_items, rows_per_item, world, p) + i0) * row_floats;
                        e = R.recv(dst, cnt * w, ncclFloat32, p, d->comm[s], (hipStream_t)streams[s]);
                        what = "ncclRecv";
                    }
                } else {
                    const size_t c = rows_count(total_items, rows_per_item, world, r);
                    if (i0 >= c) continue;
                    const size_t cnt = c - i0 < slab ? c - i0 : slab;
                    const float* src = half ? pack[s] : d_local[s] + i0 * row_floats;
                    e = R.send(src, cnt * w, ncclFloat32, root, d->comm[s], (hipStream_t)streams[s]);
                    what = "ncclSend";
                }
            }
            const ncclResult_t e2 = R.group_end();
            if (e == ncclSuccess && e2 != ncclSuccess) {
                e = e2;
                what = "ncclGroupEnd";
            }
            if (e != ncclSuccess) st = nccl_fail(what, e);
        }
        /* 3. the root expands the half rows to their place */
        if (half && rs >= 0)
            for (int r = 0; r < world && st == VV_DSP_OK; ++r) {
                const size_t c = rows_count(total_items, rows_per_item, world, r);
                if (r == root || i0 >= c) continue;
                const size_t cnt = c - i0 < slab ? c - i0 : slab;
                dev_scope g;
                st = dev_enter(&g, d->dev[rs]);
                if (st == VV_DSP_OK)
                    st = vv_dsp_spectrogram_unpack_half_device(
                        stage + (size_t)r * slab * w, cnt, row_floats,
                        d_root_out + (rows_first(total_items, rows_per_item, world, r) + i0) * row_floats, rstream);
                st = dev_leave(&g, st);
            }
    }
    /* loopback: every read of d_local[s] ran on the root's stream, so each slot
     * stream now waits for it -- the caller may overwrite d_local[s] on
     * streams[s] right away, as on the RCCL path where the send runs on streams[s] */
    if (d->loopback && st == VV_DSP_OK)
        for (int s = 0; s < d->nslots && st == VV_DSP_OK; ++s)
            if (s != rs && vvhip_stream_wait(streams[s], rstream) != 0) st = VV_DSP_ERROR_INTERNAL;
    /* stream-ordered frees: after the last use on each stream */
    for (int s = 0; s < d->nslots; ++s)
        if (pack[s]) {
            dev_scope g;
            vv_dsp_status fs = dev_enter(&g, d->dev[s]);
            if (fs == VV_DSP_OK && vvhip_free_async(pack[s], d->loopback ? rstream : streams[s]) != 0)
                fs = VV_DSP_ERROR_INTERNAL;
            fs = dev_leave(&g, fs);
            if (st == VV_DSP_OK) st = fs;
        }
    if (stage) {
        dev_scope g;
        vv_dsp_status fs = dev_enter(&g, d->dev[rs]);
        if (fs == VV_DSP_OK && vvhip_free_async(stage, rstream) != 0) fs = VV_DSP_ERROR_INTERNAL;
        fs = dev_leave(&g, fs);
        if (st == VV_DSP_OK) st = fs;
    }
    return st;
}
