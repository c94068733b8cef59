// kle_ipc.hip -- device-to-device transport over IPC-mapped mailboxes
// (KLE_TRANSPORT=ipc; kle_ctx_enable_ipc).  Replaces the RCCL send/recv
// kernels of the halo exchanges and the allreduce by copies into the peers'
// memory (hipMemcpyAsync: copy engines, no compute-unit kernels on the
// SpMV's CUs) and stream memory operations as the signals, so nothing on the
// comm stream occupies a CU while the SpMV runs and no host thread takes part
// in an exchange.  Bootstrap (the IPC handles) goes over the context's host
// callbacks.  Reference: the VecScatter of MatMult_MPIAIJ and the
// MPI_Allreduce of KSPSolve behind kle_solver.py:35.
//
// Each rank owns one mailbox (device memory, fine-grained where the driver
// exports it): per channel and peer a data flag (the sequence number of that
// peer's last delivery) and an ack flag (the last sequence that peer has
// consumed from its slot), then the slots.  A delivery of sequence s on a
// channel: the sender's stream waits until the receiver acked s - 1 (the slot
// is free), copies into the receiver's slot and writes s into the receiver's
// data flag; the receiver's stream waits for data flag >= s, copies the slot
// out (or sums it) and writes s into the sender's ack flag.  Every rank calls
// every collective in the same order, so the per-channel sequence counters
// agree without communication.
#include <cstring>
#include <vector>

#include "kle_internal.hpp"

namespace kle {

enum IpcChannel { CH_FWD_LO = 0, CH_FWD_HI, CH_REV_LO, CH_AR, IPC_NCH };
constexpr int IPC_MAXR = 64;
constexpr size_t IPC_HDR = 8192;                     // flags (2 x 4 x 64 x 8 B = 4 KB), padded
constexpr int64_t IPC_HALO_CAP = int64_t(1) << 22;   // doubles per halo slot (32 MB)
constexpr int64_t IPC_AR_CAP = PART_STRIDE;          // doubles per allreduce slot

struct IpcFlags {
    uint64_t data[IPC_NCH][IPC_MAXR];  // [channel][sender]
    uint64_t ack[IPC_NCH][IPC_MAXR];   // [channel][receiver]
};

struct IpcState {
    char *local = nullptr;          // my mailbox
    std::vector<char *> peer;       // every rank's mailbox mapped here (peer[me] = local)
    uint64_t seq[IPC_NCH] = {};
    int nranks = 1;
    size_t bytes = 0;
    double *slot(int r, IpcChannel c) const
    {
        char *b = peer[r] + IPC_HDR;
        if (c == CH_AR) return reinterpret_cast<double *>(b) + 3 * IPC_HALO_CAP;
        return reinterpret_cast<double *>(b) + (int64_t)c * IPC_HALO_CAP;
    }
    double *ar_slot(int r, int from) const { return slot(r, CH_AR) + (int64_t)from * IPC_AR_CAP; }
    uint64_t *data_flag(int r, IpcChannel c, int sender) const
    {
        return &reinterpret_cast<IpcFlags *>(peer[r])->data[c][sender];
    }
    uint64_t *ack_flag(int r, IpcChannel c, int receiver) const
    {
        return &reinterpret_cast<IpcFlags *>(peer[r])->ack[c][receiver];
    }
};

// out[i] = sum over ranks r = 0 .. nr-1 of slot r (my own term from out
// itself), in rank order: the same value on every rank
__global__ void k_rank_sum(int64_t n, int nr, int me, const double *__restrict__ slots, int64_t cap,
                           double *__restrict__ out)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double mine = out[i];
        double s = 0.0;
        for (int r = 0; r < nr; ++r) s += r == me ? mine : slots[(int64_t)r * cap + i];
        out[i] = s;
    }
}

static int wait_ge(hipStream_t st, uint64_t *flag, uint64_t v)
{
    KLE_HIP(hipStreamWaitValue64(st, flag, v, hipStreamWaitValueGte, ~uint64_t(0)));
    return 0;
}

static int post(hipStream_t st, uint64_t *flag, uint64_t v)
{
    KLE_HIP(hipStreamWriteValue64(st, flag, v, 0));
    return 0;
}

// one delivery of n doubles from src into rank `to`'s slot of channel c
static int ipc_send(kle_ctx *c, IpcChannel ch, int to, const double *src, int64_t n, double *dst, uint64_t s,
                    hipStream_t st)
{
    IpcState &P = *c->ipc;
    KLE_TRY(wait_ge(st, P.ack_flag(c->rank, ch, to), s - 1));  // the receiver has consumed s - 1
    if (n) KLE_HIP(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    return post(st, P.data_flag(to, ch, c->rank), s);
}

// the matching receive: n doubles from rank `from` out of my slot into dst
static int ipc_recv(kle_ctx *c, IpcChannel ch, int from, double *dst, int64_t n, uint64_t s, hipStream_t st)
{
    IpcState &P = *c->ipc;
    KLE_TRY(wait_ge(st, P.data_flag(c->rank, ch, from), s));
    if (n) KLE_HIP(hipMemcpyAsync(dst, P.slot(c->rank, ch), sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    return post(st, P.ack_flag(from, ch, c->rank), s);
}

int ipc_halo(kle_ctx *c, double *base, int64_t ghost_lo, int64_t n_local, int64_t ghost_hi, int lo_rank,
             int hi_rank, int64_t send_lo, int64_t send_hi, hipStream_t st)
{
    IpcState &P = *c->ipc;
    const uint64_t s = ++P.seq[CH_FWD_LO];
    KLE_ARG(send_lo <= IPC_HALO_CAP && send_hi <= IPC_HALO_CAP, "halo of %lld entries exceeds the IPC slot",
            (long long)std::max(send_lo, send_hi));
    double *own = base + ghost_lo;
    // my lowest entries are the lower neighbour's upper ghosts (its FWD_HI
    // slot), my highest the upper neighbour's lower ghosts (its FWD_LO)
    if (lo_rank >= 0) KLE_TRY(ipc_send(c, CH_FWD_HI, lo_rank, own, send_lo, P.slot(lo_rank, CH_FWD_HI), s, st));
    if (hi_rank >= 0)
        KLE_TRY(ipc_send(c, CH_FWD_LO, hi_rank, own + n_local - send_hi, send_hi, P.slot(hi_rank, CH_FWD_LO), s, st));
    if (lo_rank >= 0) KLE_TRY(ipc_recv(c, CH_FWD_LO, lo_rank, base, ghost_lo, s, st));
    if (hi_rank >= 0) KLE_TRY(ipc_recv(c, CH_FWD_HI, hi_rank, own + n_local, ghost_hi, s, st));
    return 0;
}

int ipc_reverse(kle_ctx *c, const double *send_hi, int64_t n_send, int hi_rank, double *recv_lo, int64_t n_recv,
                int lo_rank, hipStream_t st)
{
    IpcState &P = *c->ipc;
    const uint64_t s = ++P.seq[CH_REV_LO];
    KLE_ARG(n_send <= IPC_HALO_CAP, "reverse halo of %lld entries exceeds the IPC slot", (long long)n_send);
    if (hi_rank >= 0) KLE_TRY(ipc_send(c, CH_REV_LO, hi_rank, send_hi, n_send, P.slot(hi_rank, CH_REV_LO), s, st));
    if (lo_rank >= 0) KLE_TRY(ipc_recv(c, CH_REV_LO, lo_rank, recv_lo, n_recv, s, st));
    return 0;
}

int ipc_allreduce(kle_ctx *c, double *dbuf, int n, hipStream_t st)
{
    IpcState &P = *c->ipc;
    KLE_ARG(n <= IPC_AR_CAP, "allreduce of %d doubles exceeds the IPC slot", n);
    const uint64_t s = ++P.seq[CH_AR];
    const int me = c->rank;
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) {
            KLE_TRY(wait_ge(st, P.ack_flag(me, CH_AR, q), s - 1));
            KLE_HIP(hipMemcpyAsync(P.ar_slot(q, me), dbuf, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
            KLE_TRY(post(st, P.data_flag(q, CH_AR, me), s));
        }
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) KLE_TRY(wait_ge(st, P.data_flag(me, CH_AR, q), s));
    hipLaunchKernelGGL(k_rank_sum, dim3((unsigned)std::max(1, std::min(64, (n + 255) / 256))), dim3(256), 0, st,
                       (int64_t)n, c->nranks, me, P.slot(me, CH_AR), IPC_AR_CAP, dbuf);
    KLE_HIP(hipGetLastError());
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) KLE_TRY(post(st, P.ack_flag(q, CH_AR, me), s));
    return 0;
}

void ipc_destroy(kle_ctx *c)
{
    if (!c->ipc) return;
    IpcState &P = *c->ipc;
    // every rank done with every mailbox before any is unmapped
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->hcomm.allreduce) {
        double one = 1.0;
        (void)c->hcomm.allreduce(&one, 1, c->hcomm.user);
    }
    for (int r = 0; r < (int)P.peer.size(); ++r)
        if (r != c->rank && P.peer[r]) (void)hipIpcCloseMemHandle(P.peer[r]);
    if (P.local) (void)hipFree(P.local);
    delete c->ipc;
    c->ipc = nullptr;
}

}  // namespace kle

using namespace kle;

int kle_ctx_enable_ipc(kle_ctx *c)
{
    KLE_ARG(c, "null ctx");
    KLE_ARG(!c->comm && c->hcomm.allreduce, "the IPC transport bootstraps over a host-comm context");
    KLE_ARG(c->nranks <= IPC_MAXR, "at most %d ranks", IPC_MAXR);
    if (c->ipc || c->nranks == 1) return 0;
    int wait_ok = 0;
    KLE_HIP(hipDeviceGetAttribute(&wait_ok, hipDeviceAttributeCanUseStreamWaitValue, c->device));
    int bad = wait_ok ? 0 : 1;
    auto *P = new IpcState;
    P->nranks = c->nranks;
    P->bytes = IPC_HDR + sizeof(double) * (3 * IPC_HALO_CAP + (int64_t)c->nranks * IPC_AR_CAP);
    hipIpcMemHandle_t h{};
    if (!bad) {
        if (hipExtMallocWithFlags(reinterpret_cast<void **>(&P->local), P->bytes, hipDeviceMallocFinegrained) !=
                hipSuccess ||
            hipIpcGetMemHandle(&h, P->local) != hipSuccess) {
            (void)hipGetLastError();
            if (P->local) (void)hipFree(P->local);
            P->local = nullptr;
            bad = hipMalloc(reinterpret_cast<void **>(&P->local), P->bytes) != hipSuccess ||
                  hipIpcGetMemHandle(&h, P->local) != hipSuccess;
            (void)hipGetLastError();
        }
        if (!bad && hipMemset(P->local, 0, IPC_HDR) != hipSuccess) bad = 1;
    }
    // all-gather of the handles over the host callbacks: one byte per
    // double, one-hot sums (exact), plus every rank's failure flag
    const int hb = (int)sizeof(hipIpcMemHandle_t);
    std::vector<double> buf((size_t)c->nranks * (hb + 1), 0.0);
    const unsigned char *hp = reinterpret_cast<const unsigned char *>(&h);
    for (int k = 0; k < hb; ++k) buf[(size_t)c->rank * (hb + 1) + k] = hp[k];
    buf[(size_t)c->rank * (hb + 1) + hb] = bad;
    if (c->hcomm.allreduce(buf.data(), (int)buf.size(), c->hcomm.user)) {
        if (P->local) (void)hipFree(P->local);
        delete P;
        return fail(KLE_ERR_COMM, "IPC bootstrap: host allreduce failed");
    }
    int any_bad = 0;
    for (int r = 0; r < c->nranks; ++r) any_bad |= buf[(size_t)r * (hb + 1) + hb] != 0.0;
    P->peer.assign(c->nranks, nullptr);
    P->peer[c->rank] = P->local;
    for (int r = 0; r < c->nranks && !any_bad; ++r) {
        if (r == c->rank) continue;
        hipIpcMemHandle_t ph{};
        unsigned char *pp = reinterpret_cast<unsigned char *>(&ph);
        for (int k = 0; k < hb; ++k) pp[k] = (unsigned char)buf[(size_t)r * (hb + 1) + k];
        void *m = nullptr;
        if (hipIpcOpenMemHandle(&m, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            (void)hipGetLastError();
            any_bad = 1;
        }
        P->peer[r] = static_cast<char *>(m);
    }
    // agree that every rank mapped every mailbox
    double ok = any_bad ? 1.0 : 0.0;
    (void)c->hcomm.allreduce(&ok, 1, c->hcomm.user);
    if (ok != 0.0) {
        for (int r = 0; r < c->nranks; ++r)
            if (r != c->rank && P->peer[r]) (void)hipIpcCloseMemHandle(P->peer[r]);
        if (P->local) (void)hipFree(P->local);
        delete P;
        return fail(KLE_ERR_COMM, "IPC transport unavailable (stream wait-value %s, mailbox export or mapping failed "
                                  "on some rank)", wait_ok ? "supported" : "unsupported");
    }
    c->ipc = P;
    return 0;
}
