/* fake_rccl.c -- TEST INFRASTRUCTURE ONLY: a host-memory stand-in for the
 * handful of RCCL entry points vv-dsp_amd/csrc/host/dist.c resolves from
 * librccl.so.1, so dist.c's point-to-point gather branch (ncclGroupStart /
 * ncclSend / ncclRecv / ncclGroupEnd, the multi-process ncclCommInitRank form)
 * runs between 2-3 CPU processes where no two-GPU box exists
 * (tests/test_dist_rccl_sim.py).  Built with the soname librccl.so.1: loaded
 * first by path, dist.c's dlopen("librccl.so.1") then resolves to it.
 *
 * Transport: one FIFO per (sender, receiver) pair in a directory named by the
 * unique id.  Each message carries a header {magic, src, dst, count, dtype,
 * seq}; the receiver checks it against its own ncclRecv (peer, count, dtype and
 * the per-pair sequence number), so unmatched counts per (peer, slab) fail the
 * group with ncclInvalidUsage instead of passing silently.  Inside a group the
 * sends run on threads and the receives in order on the caller, so a group
 * never deadlocks on the FIFOs' buffer size.  Every completed operation is
 * appended to <dir>/ops.log ("send src dst count seq" / "recv dst src count
 * seq") for the test to compare with the schedule it expects.
 *
 * Devices and streams are not modelled here (pointers are host memory). */
#define _GNU_SOURCE
#include <rccl/rccl.h>

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#define MAXR 64
#define MAGIC 0x76766473u

struct ncclComm {
    char dir[100];
    int nranks, rank;
    int fd_out[MAXR], fd_in[MAXR];
    unsigned seq_out[MAXR], seq_in[MAXR];
};

typedef struct {
    unsigned magic, src, dst, dtype, seq, pad;
    unsigned long long count;
} msg_hdr;

typedef struct {
    int is_send;
    void* buf;
    size_t count;
    ncclDataType_t dtype;
    int peer;
    ncclComm_t comm;
    ncclResult_t res;
} op_t;

static __thread int g_depth;
static __thread op_t* g_ops;
static __thread int g_nops, g_cap;

static size_t dsize(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

static void fifo_path(char* out, size_t n, const char* dir, int src, int dst) {
    snprintf(out, n, "%s/s%d_d%d", dir, src, dst);
}

static void log_op(ncclComm_t c, const char* what, int a, int b, size_t count, unsigned seq) {
    char p[160], line[128];
    snprintf(p, sizeof p, "%s/ops.log", c->dir);
    const int fd = open(p, O_WRONLY | O_CREAT | O_APPEND, 0600);
    if (fd < 0) return;
    const int len = snprintf(line, sizeof line, "%s %d %d %zu %u\n", what, a, b, count, seq);
    if (write(fd, line, (size_t)len) != len) perror("fake_rccl: ops.log");
    close(fd);
}

static int full_io(int fd, void* buf, size_t n, int wr) {
    char* p = (char*)buf;
    while (n) {
        const ssize_t k = wr ? write(fd, p, n) : read(fd, p, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return -1;
        p += k;
        n -= (size_t)k;
    }
    return 0;
}

static int pair_fd(ncclComm_t c, int peer, int out) {
    int* fd = out ? &c->fd_out[peer] : &c->fd_in[peer];
    if (*fd >= 0) return *fd;
    char p[160];
    if (out) fifo_path(p, sizeof p, c->dir, c->rank, peer);
    else fifo_path(p, sizeof p, c->dir, peer, c->rank);
    if (mkfifo(p, 0600) != 0 && errno != EEXIST) return -1;
    *fd = open(p, out ? O_WRONLY : O_RDONLY);
    return *fd;
}

static ncclResult_t do_send(op_t* o) {
    ncclComm_t c = o->comm;
    const int fd = pair_fd(c, o->peer, 1);
    if (fd < 0) return ncclSystemError;
    msg_hdr h = {MAGIC, (unsigned)c->rank, (unsigned)o->peer, (unsigned)o->dtype, c->seq_out[o->peer]++, 0,
                 (unsigned long long)o->count};
    if (full_io(fd, &h, sizeof h, 1) || full_io(fd, o->buf, o->count * dsize(o->dtype), 1)) return ncclSystemError;
    log_op(c, "send", c->rank, o->peer, o->count, h.seq);
    return ncclSuccess;
}

static ncclResult_t do_recv(op_t* o) {
    ncclComm_t c = o->comm;
    const int fd = pair_fd(c, o->peer, 0);
    if (fd < 0) return ncclSystemError;
    msg_hdr h;
    if (full_io(fd, &h, sizeof h, 0)) return ncclSystemError;
    const unsigned want_seq = c->seq_in[o->peer]++;
    if (h.magic != MAGIC || (int)h.src != o->peer || (int)h.dst != c->rank || h.count != o->count ||
        h.dtype != (unsigned)o->dtype || h.seq != want_seq) {
        fprintf(stderr,
                "fake_rccl: rank %d recv from %d expects count %zu dtype %d seq %u, the sender posted src %u count %llu "
                "dtype %u seq %u\n",
                c->rank, o->peer, o->count, (int)o->dtype, want_seq, h.src, h.count, h.dtype, h.seq);
        /* drain the payload so the stream stays framed, then fail */
        char sink[4096];
        unsigned long long left = h.count * dsize((ncclDataType_t)h.dtype);
        while (left) {
            const size_t k = left < sizeof sink ? (size_t)left : sizeof sink;
            if (full_io(fd, sink, k, 0)) break;
            left -= k;
        }
        return ncclInvalidUsage;
    }
    if (full_io(fd, o->buf, o->count * dsize(o->dtype), 0)) return ncclSystemError;
    log_op(c, "recv", c->rank, o->peer, o->count, h.seq);
    return ncclSuccess;
}

static void* send_thread(void* arg) {
    op_t* o = (op_t*)arg;
    o->res = do_send(o);
    return NULL;
}

static ncclResult_t run_ops(op_t* ops, int n) {
    pthread_t th[256];
    int nth = 0;
    ncclResult_t r = ncclSuccess;
    for (int i = 0; i < n; ++i)
        if (ops[i].is_send) {
            if (nth == 256 || pthread_create(&th[nth], NULL, send_thread, &ops[i]) != 0) return ncclSystemError;
            ++nth;
        }
    for (int i = 0; i < n; ++i)
        if (!ops[i].is_send) {
            const ncclResult_t e = do_recv(&ops[i]);
            if (r == ncclSuccess) r = e;
        }
    for (int i = 0; i < nth; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < n; ++i)
        if (ops[i].is_send && r == ncclSuccess) r = ops[i].res;
    return r;
}

static ncclResult_t post(int is_send, void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm) {
    if (!comm || peer < 0 || peer >= comm->nranks || peer == comm->rank || !dsize(dt)) return ncclInvalidArgument;
    if (!buf && count) return ncclInvalidArgument;
    op_t o = {is_send, buf, count, dt, peer, comm, ncclSuccess};
    if (g_depth == 0) return run_ops(&o, 1);
    if (g_nops == g_cap) {
        g_cap = g_cap ? 2 * g_cap : 64;
        g_ops = (op_t*)realloc(g_ops, sizeof(op_t) * (size_t)g_cap);
        if (!g_ops) return ncclSystemError;
    }
    g_ops[g_nops++] = o;
    return ncclSuccess;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    char tmpl[] = "/tmp/fake_rccl_XXXXXX";
    if (!mkdtemp(tmpl)) return ncclSystemError;
    memset(id->internal, 0, sizeof id->internal);
    memcpy(id->internal, tmpl, strlen(tmpl));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    ncclComm_t c = (ncclComm_t)calloc(1, sizeof *c);
    if (!c) return ncclSystemError;
    memcpy(c->dir, id.internal, sizeof c->dir - 1);
    c->nranks = nranks;
    c->rank = rank;
    for (int i = 0; i < MAXR; ++i) c->fd_out[i] = c->fd_in[i] = -1;
    *comm = c;
    log_op(c, "init", rank, nranks, 0, 0);
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    (void)comms; (void)ndev; (void)devlist;
    return ncclInvalidUsage;   /* one process per rank only */
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    for (int i = 0; i < MAXR; ++i) {
        if (comm->fd_out[i] >= 0) close(comm->fd_out[i]);
        if (comm->fd_in[i] >= 0) close(comm->fd_in[i]);
    }
    free(comm);
    return ncclSuccess;
}

ncclResult_t ncclGroupStart(void) {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void) {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    const ncclResult_t r = run_ops(g_ops, g_nops);
    g_nops = 0;
    return r;
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t s) {
    (void)s;
    return post(1, (void*)buf, count, dt, peer, comm);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t s) {
    (void)s;
    return post(0, buf, count, dt, peer, comm);
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "fake: success";
        case ncclInvalidUsage: return "fake: invalid usage (unmatched send/recv)";
        case ncclInvalidArgument: return "fake: invalid argument";
        case ncclSystemError: return "fake: system error";
        default: return "fake: error";
    }
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->nranks;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
    if (!comm || !rank) return ncclInvalidArgument;
    *rank = comm->rank;
    return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
    if (!comm || !device) return ncclInvalidArgument;
    *device = 0;
    return ncclSuccess;
}
