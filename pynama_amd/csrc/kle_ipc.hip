// kle_ipc.hip -- device-to-device transport over IPC-mapped mailboxes
// (KLE_TRANSPORT=ipc; kle_ctx_enable_ipc).  Replaces the RCCL send/recv
// kernels of the halo exchanges and the allreduce by copies into the peers'
// memory (hipMemcpyAsync: copy engines, no compute-unit kernels on the
// SpMV's CUs) and stream memory operations as the signals, so nothing on the
// comm stream occupies a CU while the SpMV runs and no host thread takes part
// in an exchange.  Bootstrap (the IPC handles) goes over the context's host
// callbacks.  Reference: the VecScatter of MatMult_MPIAIJ and the
// MPI_Allreduce of KSPSolve behind kle_solver.py:35, on a slab or a Chaco
// (graph) partition (dmplex.py:21).
//
// Each rank owns one mailbox (fine-grained device memory: peers write into it
// and its own stream polls flags in it, so writes from other devices must
// become visible without a kernel boundary; a rank whose driver cannot export
// fine-grained memory refuses the transport): per channel and peer a data
// flag (the sequence number of that peer's last delivery) and an ack flag (the
// last sequence that peer has consumed from its slot), then the slots.  A
// delivery of sequence s on a channel: the sender's stream waits until the
// receiver acked s - 1 (the slot is free), copies into the receiver's slot and
// writes s into the receiver's data flag; the receiver's stream waits for data
// flag >= s, copies the slot out (or sums it) and writes s into the sender's
// ack flag.  The sequence numbers count per channel AND per ordered pair
// (sender -> receiver): a rank whose halo plan has no peers skips the
// exchange, and only the pairs that exchange advance, so any later plan that
// pairs it with a peer finds both counters in step.
//
// Slab partitions use one slot per direction (FWD_LO / FWD_HI / REV_LO);
// graph partitions (HaloPlan: any number of peers) and the allreduce use one
// slot per sender.
//
// Deadline: a peer that dies or stops calling the collectives leaves this
// rank's stream waiting on a flag forever (a stream wait has no timeout).
// Every collective therefore ends with a stream write of its ticket into a
// host-pinned progress word, and a watchdog thread watches the issued tickets.
// When one makes no progress it checks the processes of the peers that
// collective waits on (pids and process start times are exchanged at
// bootstrap): a peer that has exited -- or whose pid now names a later
// process -- ends this process after IPC_DEAD_GRACE_S.  A peer this process
// cannot see with the start time it reported (another PID namespace) gets no
// such check.
// A live peer doing long host-only work between collectives (I/O, CPU
// assembly) is never cut off -- as with NCCL, operations have no timeout --
// unless KLE_COMM_TIMEOUT_S > 0 sets one.  The exit status is KLE_IPC_EXIT
// (75): the host thread is blocked inside the runtime and cannot return an
// error, and a process exit is what frees the stuck queue.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

#include "kle_internal.hpp"

namespace kle {

enum IpcChannel { CH_FWD_LO = 0, CH_FWD_HI, CH_REV_LO, CH_AR, CH_PFWD, CH_PREV, IPC_NCH };
static const char *const ch_name[IPC_NCH] = {"halo (to lower)", "halo (to upper)", "reverse halo", "allreduce",
                                              "plan halo", "plan reverse halo"};
constexpr int IPC_MAXR = 64;
constexpr size_t IPC_HDR = 16384;                    // flags (2 x 6 x 64 x 8 B = 6 KB), padded
constexpr int64_t IPC_HALO_CAP = int64_t(1) << 22;   // doubles per slab halo slot (32 MB)
constexpr int64_t IPC_AR_CAP = PART_STRIDE;          // doubles per allreduce slot (one per sender)
constexpr int64_t IPC_PLAN_CAP = int64_t(1) << 19;   // doubles per graph-halo slot (4 MB, one per sender)
constexpr int KLE_IPC_EXIT = 75;                     // process exit status of a missed deadline
constexpr double IPC_DEAD_GRACE_S = 2.0;             // stalled this long with an awaited peer gone: exit

struct IpcFlags {
    uint64_t data[IPC_NCH][IPC_MAXR];  // [channel][sender]
    uint64_t ack[IPC_NCH][IPC_MAXR];   // [channel][receiver]
};
static_assert(sizeof(IpcFlags) <= IPC_HDR, "mailbox header");

struct IpcState {
    char *local = nullptr;          // my mailbox
    std::vector<char *> peer;       // every rank's mailbox mapped here (peer[me] = local)
    std::vector<long> pid;          // every rank's process id (bootstrap)
    std::vector<long long> pstart;  // its start time as seen here (-1: not visible, no dead-peer check)
    uint64_t sseq[IPC_NCH][IPC_MAXR] = {};  // deliveries sent to each rank, per channel
    uint64_t rseq[IPC_NCH][IPC_MAXR] = {};  // deliveries received from each rank, per channel
    int nranks = 1;
    size_t bytes = 0;
    // watchdog: progress words per stream (0 compute, 1 comm), host-pinned,
    // written by the GPU after each collective; issued tickets and what the
    // newest collective on each stream was waiting for
    volatile uint64_t *h_prog = nullptr;
    uint64_t *d_prog = nullptr;
    std::atomic<uint64_t> issued[2];
    std::mutex mu;
    std::string what[2];
    std::vector<int> awaited[2];    // peers of the newest collective per stream
    std::thread wd;
    std::atomic<bool> stop{false};
    double deadline_s = 0.0;        // > 0: also exit on a live peer's stall (KLE_COMM_TIMEOUT_S)
    int rank = 0;

    IpcState() { issued[0] = issued[1] = 0; }
    double *region(int r, IpcChannel c) const
    {
        double *b = reinterpret_cast<double *>(peer[r] + IPC_HDR);
        if (c <= CH_REV_LO) return b + (int64_t)c * IPC_HALO_CAP;
        b += 3 * IPC_HALO_CAP;
        if (c == CH_AR) return b;
        b += (int64_t)nranks * IPC_AR_CAP;
        return b + (c == CH_PFWD ? 0 : (int64_t)nranks * IPC_PLAN_CAP);
    }
    double *slot(int r, IpcChannel c) const { return region(r, c); }  // slab channels: one slot
    double *ar_slot(int r, int from) const { return region(r, CH_AR) + (int64_t)from * IPC_AR_CAP; }
    double *plan_slot(int r, IpcChannel c, int from) const { return region(r, c) + (int64_t)from * IPC_PLAN_CAP; }
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
// The peers' slots are read at system scope: their copies land in this
// rank's fine-grained mailbox from other processes (copy engines, other
// XCDs' caches), and a plain load may return the line this kernel's
// previous launch left in its L2 -- last iteration's partials (a rare
// stale sum, seen as a NaN in an 8-rank pipelined CG on one GPU).
// Sentinel (tuning ipc_sentinel, a debug mode the multirank tests run once):
// every consumed slot entry is overwritten with NaN at system scope before the
// ack goes out, so a read of a slot the peer has not refilled for this
// sequence -- too early, or a stale line of this GPU's L2 (which the
// write-through NaN store updates too) -- yields NaN at once instead of last
// iteration's finite value.
__global__ void k_rank_sum(int64_t n, int nr, int me, double *__restrict__ slots, int64_t cap,
                           double *__restrict__ out, int sentinel)
{
    const double qnan = __builtin_nan("");
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double mine = out[i];
        double s = 0.0;
        for (int r = 0; r < nr; ++r)
            s += r == me ? mine
                         : __hip_atomic_load(slots + (int64_t)r * cap + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        out[i] = s;
        if (sentinel)
            for (int r = 0; r < nr; ++r)
                if (r != me)
                    __hip_atomic_store(slots + (int64_t)r * cap + i, qnan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// A slot out of this rank's mailbox at system scope (k_rank_sum's reason)
__global__ void k_slot_copy(int64_t n, double *__restrict__ src, double *__restrict__ dst, int sentinel)
{
    const double qnan = __builtin_nan("");
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (sentinel) __hip_atomic_store(src + i, qnan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// the end of one collective on stream st: its ticket into the progress word
// the watchdog reads (and what it was, for the report)
static int ipc_done(kle_ctx *c, hipStream_t st, IpcChannel ch, const std::vector<int> &peers)
{
    IpcState &P = *c->ipc;
    const int k = st == c->comm_stream ? 1 : 0;
    {
        std::string w = std::string(ch_name[ch]) + " with rank(s)";
        for (int q : peers) w += " " + std::to_string(q);
        std::lock_guard<std::mutex> lk(P.mu);
        P.what[k] = w;
        P.awaited[k] = peers;
    }
    return post(st, P.d_prog + k, ++P.issued[k]);
}

// A process's start time (field 22 of /proc/<pid>/stat, clock ticks after
// boot) and state letter; -1 when /proc does not show it here
static long long proc_start(long pid, char *state)
{
    char path[64];
    snprintf(path, sizeof path, "/proc/%ld/stat", pid);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char buf[1024];
    const size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *e = strrchr(buf, ')');  // (the fields follow the command name)
    if (!e || e[1] != ' ') return -1;
    if (state) *state = e[2];
    const char *q = e + 2;  // field 3 (state)
    for (int fld = 3; fld < 22 && *q; ++fld) {
        q = strchr(q, ' ');
        if (!q) return -1;
        ++q;
    }
    return *q ? atoll(q) : -1;
}

// has process pid (started at start) ended?  Gone from /proc, a zombie not
// yet reaped, or the pid reused by a later process.  Only for peers whose
// pid and start time this process saw at bootstrap: ranks in other PID
// namespaces (IPC allows containers that share --ipc=host but not --pid)
// are never taken for dead -- for them only KLE_COMM_TIMEOUT_S applies.
static bool pid_dead(long pid, long long start)
{
    if (pid <= 0 || start < 0) return false;  // (not verifiable from here)
    char st = 0;
    const long long s = proc_start(pid, &st);
    return s < 0 || s != start || st == 'Z' || st == 'X';
}

static void ipc_watchdog(IpcState *P)
{
    using clk = std::chrono::steady_clock;
    uint64_t seen[2] = {P->h_prog[0], P->h_prog[1]};
    clk::time_point since[2] = {clk::now(), clk::now()};
    while (!P->stop.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        for (int k = 0; k < 2; ++k) {
            const uint64_t done = P->h_prog[k], iss = P->issued[k].load();
            if (done >= iss || done != seen[k]) {
                seen[k] = done;
                since[k] = clk::now();
                continue;
            }
            const double idle = std::chrono::duration<double>(clk::now() - since[k]).count();
            if (idle < IPC_DEAD_GRACE_S) continue;
            std::string w;
            int gone = -1;
            {
                std::lock_guard<std::mutex> lk(P->mu);
                w = P->what[k];
                for (int q : P->awaited[k])
                    if (q >= 0 && q < (int)P->pid.size() && pid_dead(P->pid[q], P->pstart[q])) gone = q;
            }
            if (gone < 0 && !(P->deadline_s > 0.0 && idle > P->deadline_s)) continue;
            if (gone >= 0)
                fprintf(stderr,
                        "kle: rank %d: IPC transport stalled %.0f s on the %s stream (collective %llu of %llu; newest: "
                        "%s) and rank %d (pid %ld) has exited -- exiting with status %d\n",
                        P->rank, idle, k ? "comm" : "compute", (unsigned long long)done + 1, (unsigned long long)iss,
                        w.c_str(), gone, P->pid[gone], KLE_IPC_EXIT);
            else
                fprintf(stderr,
                        "kle: rank %d: IPC transport made no progress for %.0f s on the %s stream (collective %llu of "
                        "%llu; newest: %s): a peer stopped calling the collectives (KLE_COMM_TIMEOUT_S) -- exiting "
                        "with status %d\n",
                        P->rank, idle, k ? "comm" : "compute", (unsigned long long)done + 1,
                        (unsigned long long)iss, w.c_str(), KLE_IPC_EXIT);
            fflush(stderr);
            _exit(KLE_IPC_EXIT);
        }
    }
}

// one delivery of n doubles from src into dst (rank `to`'s slot of channel c),
// the pair's next sequence number
static int ipc_send(kle_ctx *c, IpcChannel ch, int to, const double *src, int64_t n, double *dst, hipStream_t st)
{
    IpcState &P = *c->ipc;
    const uint64_t s = ++P.sseq[ch][to];
    KLE_TRY(wait_ge(st, P.ack_flag(c->rank, ch, to), s - 1));  // the receiver has consumed s - 1
    if (n) KLE_HIP(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    return post(st, P.data_flag(to, ch, c->rank), s);
}

// the matching receive: n doubles from rank `from` out of src (my slot) into dst
static int ipc_recv(kle_ctx *c, IpcChannel ch, int from, double *dst, double *src, int64_t n, hipStream_t st)
{
    IpcState &P = *c->ipc;
    const uint64_t s = ++P.rseq[ch][from];
    KLE_TRY(wait_ge(st, P.data_flag(c->rank, ch, from), s));
    if (n) {
        hipLaunchKernelGGL(k_slot_copy, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(256, (n + 255) / 256))),
                           dim3(256), 0, st, n, src, dst, g_tune.ipc_sentinel);
        KLE_HIP(hipGetLastError());
    }
    return post(st, P.ack_flag(from, ch, c->rank), s);
}

int ipc_halo(kle_ctx *c, double *base, int64_t ghost_lo, int64_t n_local, int64_t ghost_hi, int lo_rank,
             int hi_rank, int64_t send_lo, int64_t send_hi, hipStream_t st)
{
    IpcState &P = *c->ipc;
    // (sizes checked before the sequence moves: a refused call leaves the
    // counters in step with the peers')
    KLE_ARG(send_lo <= IPC_HALO_CAP && send_hi <= IPC_HALO_CAP && ghost_lo <= IPC_HALO_CAP &&
                ghost_hi <= IPC_HALO_CAP,
            "halo of %lld entries exceeds the IPC slot",
            (long long)std::max(std::max(send_lo, send_hi), std::max(ghost_lo, ghost_hi)));
    double *own = base + ghost_lo;
    // my lowest entries are the lower neighbour's upper ghosts (its FWD_HI
    // slot), my highest the upper neighbour's lower ghosts (its FWD_LO)
    if (lo_rank >= 0) KLE_TRY(ipc_send(c, CH_FWD_HI, lo_rank, own, send_lo, P.slot(lo_rank, CH_FWD_HI), st));
    if (hi_rank >= 0)
        KLE_TRY(ipc_send(c, CH_FWD_LO, hi_rank, own + n_local - send_hi, send_hi, P.slot(hi_rank, CH_FWD_LO), st));
    if (lo_rank >= 0) KLE_TRY(ipc_recv(c, CH_FWD_LO, lo_rank, base, P.slot(c->rank, CH_FWD_LO), ghost_lo, st));
    if (hi_rank >= 0)
        KLE_TRY(ipc_recv(c, CH_FWD_HI, hi_rank, own + n_local, P.slot(c->rank, CH_FWD_HI), ghost_hi, st));
    std::vector<int> pr;
    if (lo_rank >= 0) pr.push_back(lo_rank);
    if (hi_rank >= 0) pr.push_back(hi_rank);
    return ipc_done(c, st, CH_FWD_LO, pr);
}

int ipc_reverse(kle_ctx *c, const double *send_hi, int64_t n_send, int hi_rank, double *recv_lo, int64_t n_recv,
                int lo_rank, hipStream_t st)
{
    IpcState &P = *c->ipc;
    KLE_ARG(n_send <= IPC_HALO_CAP && n_recv <= IPC_HALO_CAP, "reverse halo of %lld entries exceeds the IPC slot",
            (long long)std::max(n_send, n_recv));
    if (hi_rank >= 0) KLE_TRY(ipc_send(c, CH_REV_LO, hi_rank, send_hi, n_send, P.slot(hi_rank, CH_REV_LO), st));
    if (lo_rank >= 0) KLE_TRY(ipc_recv(c, CH_REV_LO, lo_rank, recv_lo, P.slot(c->rank, CH_REV_LO), n_recv, st));
    std::vector<int> pr;
    if (lo_rank >= 0) pr.push_back(lo_rank);
    if (hi_rank >= 0) pr.push_back(hi_rank);
    return ipc_done(c, st, CH_REV_LO, pr);
}

// Graph-partition halo (HaloPlan): sbuf holds the packed sends (peer k's
// slice at send_off[k] * bs); each peer's ghost group lands in place at ext
// node recv_off[k].  The plans are symmetric (kle_umesh.cpp: a rank sends to
// exactly the ranks it receives from), so every pair delivers at every call.
int ipc_halo_plan(kle_ctx *c, double *base, const HaloPlan &H, int bs, const double *sbuf, hipStream_t st)
{
    IpcState &P = *c->ipc;
    const size_t np = H.peers.size();
    for (size_t k = 0; k < np; ++k)
        KLE_ARG(H.send_cnt[k] * bs <= IPC_PLAN_CAP && H.recv_cnt[k] * bs <= IPC_PLAN_CAP,
                "graph halo of %lld entries (rank %d) exceeds the IPC slot",
                (long long)(std::max(H.send_cnt[k], H.recv_cnt[k]) * bs), H.peers[k]);
    const int me = c->rank;
    for (size_t k = 0; k < np; ++k) {
        const int q = H.peers[k];
        KLE_TRY(ipc_send(c, CH_PFWD, q, sbuf + H.send_off[k] * bs, H.send_cnt[k] * bs, P.plan_slot(q, CH_PFWD, me), st));
    }
    for (size_t k = 0; k < np; ++k) {
        const int q = H.peers[k];
        KLE_TRY(ipc_recv(c, CH_PFWD, q, base + H.recv_off[k] * bs, P.plan_slot(me, CH_PFWD, q), H.recv_cnt[k] * bs,
                         st));
    }
    return ipc_done(c, st, CH_PFWD, H.peers);
}

// Reverse of a graph-partition halo (halo_reverse_plan's transfer): to each
// higher peer the sums of its ghost group (gsend from ext node hi0 on), from
// each lower peer its sums for the owned nodes of my send slice to it (rbuf).
int ipc_reverse_plan(kle_ctx *c, const HaloPlan &H, int64_t hi0, int bs, const double *gsend, double *rbuf,
                     hipStream_t st)
{
    IpcState &P = *c->ipc;
    const size_t np = H.peers.size();
    const int me = c->rank;
    for (size_t k = 0; k < np; ++k)
        KLE_ARG(H.send_cnt[k] * bs <= IPC_PLAN_CAP && H.recv_cnt[k] * bs <= IPC_PLAN_CAP,
                "reverse graph halo of %lld entries (rank %d) exceeds the IPC slot",
                (long long)(std::max(H.send_cnt[k], H.recv_cnt[k]) * bs), H.peers[k]);
    for (size_t k = 0; k < np; ++k) {
        const int q = H.peers[k];
        if (q > me)
            KLE_TRY(ipc_send(c, CH_PREV, q, gsend + (H.recv_off[k] - hi0) * bs, H.recv_cnt[k] * bs,
                             P.plan_slot(q, CH_PREV, me), st));
    }
    for (size_t k = 0; k < np; ++k) {
        const int q = H.peers[k];
        if (q < me)
            KLE_TRY(ipc_recv(c, CH_PREV, q, rbuf + H.send_off[k] * bs, P.plan_slot(me, CH_PREV, q), H.send_cnt[k] * bs,
                             st));
    }
    return ipc_done(c, st, CH_PREV, H.peers);
}

int ipc_allreduce(kle_ctx *c, double *dbuf, int n, hipStream_t st)
{
    IpcState &P = *c->ipc;
    KLE_ARG(n <= IPC_AR_CAP, "allreduce of %d doubles exceeds the IPC slot", n);
    const int me = c->rank;
    std::vector<int> pr;
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) {
            pr.push_back(q);
            const uint64_t s = ++P.sseq[CH_AR][q];
            KLE_TRY(wait_ge(st, P.ack_flag(me, CH_AR, q), s - 1));
            KLE_HIP(hipMemcpyAsync(P.ar_slot(q, me), dbuf, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
            KLE_TRY(post(st, P.data_flag(q, CH_AR, me), s));
        }
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) KLE_TRY(wait_ge(st, P.data_flag(me, CH_AR, q), ++P.rseq[CH_AR][q]));
    hipLaunchKernelGGL(k_rank_sum, dim3((unsigned)std::max(1, std::min(64, (n + 255) / 256))), dim3(256), 0, st,
                       (int64_t)n, c->nranks, me, P.region(me, CH_AR), IPC_AR_CAP, dbuf, g_tune.ipc_sentinel);
    KLE_HIP(hipGetLastError());
    for (int q = 0; q < c->nranks; ++q)
        if (q != me) KLE_TRY(post(st, P.ack_flag(q, CH_AR, me), P.rseq[CH_AR][q]));
    return ipc_done(c, st, CH_AR, pr);
}

static void ipc_free(IpcState *P, int me, bool unmap)
{
    if (P->wd.joinable()) {
        P->stop = true;
        P->wd.join();
    }
    if (unmap) {
        for (int r = 0; r < (int)P->peer.size(); ++r)
            if (r != me && P->peer[r]) (void)hipIpcCloseMemHandle(P->peer[r]);
        if (P->local) (void)hipFree(P->local);
    }
    if (P->h_prog) (void)hipHostFree((void *)P->h_prog);
    delete P;
}

void ipc_destroy(kle_ctx *c)
{
    if (!c->ipc) return;
    // every rank done with every mailbox before any is unmapped (the watchdog
    // still guards these synchronisations)
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    bool barrier = false;
    if (c->hcomm.allreduce) {
        double one = 1.0;
        barrier = c->hcomm.allreduce(&one, 1, c->hcomm.user) == 0;
    }
    // without the barrier a peer may still be writing its last acks into my
    // mailbox: keep it (and my mappings of theirs) rather than free memory in use
    ipc_free(c->ipc, c->rank, barrier);
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
    const char *why = wait_ok ? "" : "stream wait-value unsupported";
    auto *P = new IpcState;
    P->nranks = c->nranks;
    P->rank = c->rank;
    if (const char *e = getenv("KLE_COMM_TIMEOUT_S"))
        if (atof(e) > 0) P->deadline_s = atof(e);
    P->bytes = IPC_HDR + sizeof(double) * (3 * IPC_HALO_CAP + (int64_t)c->nranks * (IPC_AR_CAP + 2 * IPC_PLAN_CAP));
    hipIpcMemHandle_t h{};
    if (!bad) {
        // fine-grained or nothing: peers on other devices write flags and
        // data that this rank's stream polls without a kernel boundary
        if (hipExtMallocWithFlags(reinterpret_cast<void **>(&P->local), P->bytes, hipDeviceMallocFinegrained) !=
                hipSuccess ||
            hipIpcGetMemHandle(&h, P->local) != hipSuccess) {
            (void)hipGetLastError();
            bad = 1;
            why = "fine-grained mailbox allocation or export failed";
        } else if (hipMemset(P->local, 0, IPC_HDR) != hipSuccess) {
            bad = 1;
            why = "mailbox clear failed";
        }
    }
    // the watchdog's progress words: host-pinned, written by the GPU; one
    // write checked here so a driver that cannot target them refuses at once
    void *hp = nullptr;
    if (!bad) {
        if (hipHostMalloc(&hp, 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void **>(&P->d_prog), hp, 0) != hipSuccess) {
            (void)hipGetLastError();
            bad = 1;
            why = "pinned progress word allocation failed";
        } else {
            P->h_prog = static_cast<volatile uint64_t *>(hp);
            P->h_prog[0] = P->h_prog[1] = 0;
            if (hipStreamWriteValue64(c->stream, P->d_prog, 7, 0) != hipSuccess ||
                hipStreamSynchronize(c->stream) != hipSuccess || P->h_prog[0] != 7) {
                (void)hipGetLastError();
                bad = 1;
                why = "stream write-value into pinned host memory failed";
            }
            P->h_prog[0] = 0;
        }
    }
    // all-gather of the handles over the host callbacks: one byte per
    // double, one-hot sums (exact), plus every rank's failure flag and pid
    const int hb = (int)sizeof(hipIpcMemHandle_t), hs = hb + 3;
    std::vector<double> buf((size_t)c->nranks * hs, 0.0);
    const unsigned char *hpb = reinterpret_cast<const unsigned char *>(&h);
    for (int k = 0; k < hb; ++k) buf[(size_t)c->rank * hs + k] = hpb[k];
    buf[(size_t)c->rank * hs + hb] = bad;
    buf[(size_t)c->rank * hs + hb + 1] = (double)getpid();
    buf[(size_t)c->rank * hs + hb + 2] = (double)proc_start((long)getpid(), nullptr);  // (< 2^53: exact)
    if (c->hcomm.allreduce(buf.data(), (int)buf.size(), c->hcomm.user)) {
        ipc_free(P, c->rank, true);
        return fail(KLE_ERR_COMM, "IPC bootstrap: host allreduce failed");
    }
    int any_bad = 0;
    P->pid.assign(c->nranks, 0);
    P->pstart.assign(c->nranks, -1);
    for (int r = 0; r < c->nranks; ++r) {
        any_bad |= buf[(size_t)r * hs + hb] != 0.0;
        P->pid[r] = (long)buf[(size_t)r * hs + hb + 1];
        // (the dead-peer check only for a peer whose pid this process sees
        // with the start time that peer reported: same PID namespace)
        const long long st = (long long)buf[(size_t)r * hs + hb + 2];
        if (st >= 0 && proc_start(P->pid[r], nullptr) == st) P->pstart[r] = st;
    }
    P->peer.assign(c->nranks, nullptr);
    P->peer[c->rank] = P->local;
    for (int r = 0; r < c->nranks && !any_bad; ++r) {
        if (r == c->rank) continue;
        hipIpcMemHandle_t ph{};
        unsigned char *pp = reinterpret_cast<unsigned char *>(&ph);
        for (int k = 0; k < hb; ++k) pp[k] = (unsigned char)buf[(size_t)r * hs + k];
        void *m = nullptr;
        if (hipIpcOpenMemHandle(&m, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            (void)hipGetLastError();
            any_bad = 1;
            why = "mapping a peer's mailbox failed";
        }
        P->peer[r] = static_cast<char *>(m);
    }
    // agree that every rank mapped every mailbox
    double ok = any_bad ? 1.0 : 0.0;
    (void)c->hcomm.allreduce(&ok, 1, c->hcomm.user);
    if (ok != 0.0) {
        ipc_free(P, c->rank, true);
        return fail(KLE_ERR_COMM, "IPC transport unavailable on some rank (here: %s)", *why ? why : "ok");
    }
    P->wd = std::thread(ipc_watchdog, P);
    c->ipc = P;
    return 0;
}
