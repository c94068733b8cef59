"""Process-level runtime: one kle context (HIP device + stream + RCCL comm)
per process, one process per GPU.

Rank/world come from torch.distributed when it is initialised (torchrun sets
RANK / LOCAL_RANK / WORLD_SIZE), otherwise from the environment, otherwise a
single rank.  The RCCL unique id is made on rank 0 by libkle and broadcast
over torch.distributed -- PyTorch is only the bootstrap here.
"""
import ctypes as C
import os
import sys

from ._lib import ALLREDUCE_FN, EXCHANGE_FN, HALO_FN, HostComm, call, load


def _dist():
    # import torch only when a multi-rank launch can have initialised it
    if "torch" not in sys.modules and int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:  # torch absent or broken: single rank
        pass
    return None


def world():
    """(rank, size) without touching the GPU."""
    d = _dist()
    if d is not None:
        return d.get_rank(), d.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


class Comm:
    """petsc4py COMM_WORLD stand-in: rank / size, and tompi4py() -> the same
    object with the mpi4py calls the reference's host code makes on it
    (allgather of Python objects, boundary_conditions.py:201,221,233,271),
    over torch.distributed (gloo / RCCL process group) when one is
    initialised, else a one-rank world."""

    @property
    def rank(self):
        return world()[0]

    @property
    def size(self):
        return world()[1]

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def tompi4py(self):
        return self

    def allgather(self, obj):
        """mpi4py Comm.allgather: every rank's obj, in rank order."""
        d = _dist()
        if d is None or d.get_world_size() == 1:
            return [obj]
        out = [None] * d.get_world_size()
        d.all_gather_object(out, obj)
        return out

    def bcast(self, obj, root=0):
        """mpi4py Comm.bcast: root's obj on every rank."""
        d = _dist()
        if d is None or d.get_world_size() == 1:
            return obj
        box = [obj if d.get_rank() == root else None]
        d.broadcast_object_list(box, src=root)
        return box[0]

    def barrier(self):
        ctx = get_ctx()
        call("kle_ctx_barrier", ctx.h)


COMM_WORLD = Comm()


class Context:
    """transport: "rccl" (default, one GPU per rank), "host" (collectives
    staged through host memory over torch.distributed/gloo; several ranks may
    share one GPU -- used to test the distributed path on a single device) or
    "ipc" (halos and allreduces as copies into IPC-mapped peer mailboxes with
    stream wait/write-value signals, bootstrapped over gloo;
    kle_ctx_enable_ipc -- several ranks may share one GPU as well).
    KLE_RCCL_SELF=1 on a single rank creates a one-rank RCCL communicator, so
    the RCCL calls (init with deadline, allreduce on both streams) run on one
    GPU; RCCL refuses two ranks on one device."""

    def __init__(self, device=None, rank=None, nranks=None, transport=None):
        load()
        r, n = world()
        self.rank = r if rank is None else rank
        self.nranks = n if nranks is None else nranks
        self.transport = transport or os.environ.get("KLE_TRANSPORT", "rccl")
        if device is None:
            default = 0 if self.transport == "host" else (self.rank if self.nranks > 1 else 0)
            device = int(os.environ.get("KLE_DEVICE", os.environ.get("LOCAL_RANK", default)))
            if self.transport == "host":
                device = int(os.environ.get("KLE_DEVICE", 0))
            elif self.transport == "ipc":  # one GPU per rank under torchrun, else all on 0 (tests)
                device = int(os.environ.get("KLE_DEVICE", os.environ.get("LOCAL_RANK", 0)))
        self.device = device
        h = C.c_void_p()
        if self.nranks > 1 and self.transport in ("host", "ipc"):
            self._hc = self._host_comm()
            call("kle_ctx_create_host_comm", device, self.rank, self.nranks, C.byref(self._hc), C.byref(h))
            if self.transport == "ipc":
                try:
                    call("kle_ctx_enable_ipc", h)
                except Exception:
                    call("kle_ctx_destroy", h)
                    raise
        else:
            if self.nranks > 1:
                uid = self._bcast_unique_id()
            elif os.environ.get("KLE_RCCL_SELF") == "1":
                # a one-rank RCCL communicator: the solver's collectives run
                # through RCCL on one GPU (tests of the RCCL transport)
                raw = C.create_string_buffer(128)
                call("kle_get_unique_id", raw)
                uid = bytes(raw.raw)
            else:
                uid = None
            call("kle_ctx_create", device, self.rank, self.nranks, uid, C.byref(h))
        self.h = h

    def _host_comm(self):
        import numpy as np
        import torch
        d = _dist()
        if d is None:
            raise RuntimeError("host transport needs torch.distributed initialised")

        def allreduce(buf, n, user):
            try:
                a = np.ctypeslib.as_array(buf, (n,))
                t = torch.from_numpy(a.copy())
                d.all_reduce(t)
                a[:] = t.numpy()
                return 0
            except Exception:
                return 1

        def halo(s_lo, n_slo, lo_rank, s_hi, n_shi, hi_rank, r_lo, n_rlo, r_hi, n_rhi, user):
            try:
                reqs, bufs = [], []
                if lo_rank >= 0:
                    if n_slo:
                        reqs.append(d.isend(torch.from_numpy(np.ctypeslib.as_array(s_lo, (n_slo,)).copy()), lo_rank))
                    if n_rlo:
                        t = torch.zeros(n_rlo, dtype=torch.float64)
                        reqs.append(d.irecv(t, lo_rank))
                        bufs.append((r_lo, n_rlo, t))
                if hi_rank >= 0:
                    if n_shi:
                        reqs.append(d.isend(torch.from_numpy(np.ctypeslib.as_array(s_hi, (n_shi,)).copy()), hi_rank))
                    if n_rhi:
                        t = torch.zeros(n_rhi, dtype=torch.float64)
                        reqs.append(d.irecv(t, hi_rank))
                        bufs.append((r_hi, n_rhi, t))
                for q in reqs:
                    q.wait()
                for ptr, n, t in bufs:
                    np.ctypeslib.as_array(ptr, (n,))[:] = t.numpy()
                return 0
            except Exception:
                return 1

        def exchange(npeers, peers, send, scnt, recv, rcnt, user):
            # graph-partition halo: packed per-peer slices, peer order
            try:
                reqs, bufs, so, ro = [], [], 0, 0
                for k in range(npeers):
                    q, ns, nr = peers[k], scnt[k], rcnt[k]
                    if ns:
                        reqs.append(d.isend(torch.from_numpy(np.ctypeslib.as_array(send, (so + ns,))[so:].copy()), q))
                    if nr:
                        t = torch.zeros(nr, dtype=torch.float64)
                        reqs.append(d.irecv(t, q))
                        bufs.append((ro, nr, t))
                    so += ns
                    ro += nr
                for r in reqs:
                    r.wait()
                if ro:
                    out = np.ctypeslib.as_array(recv, (ro,))
                    for o, n, t in bufs:
                        out[o:o + n] = t.numpy()
                return 0
            except Exception:
                return 1

        self._cb = (ALLREDUCE_FN(allreduce), HALO_FN(halo), EXCHANGE_FN(exchange))
        return HostComm(self._cb[0], self._cb[1], None, self._cb[2])

    def _bcast_unique_id(self):
        d = _dist()
        if d is None:
            raise RuntimeError("nranks > 1 needs torch.distributed initialised for the RCCL bootstrap")
        buf = [None]
        if self.rank == 0:
            raw = C.create_string_buffer(128)
            call("kle_get_unique_id", raw)
            buf[0] = bytes(raw.raw)
        d.broadcast_object_list(buf, src=0)
        return buf[0]

    def synchronize(self):
        call("kle_ctx_synchronize", self.h)

    def barrier(self):
        call("kle_ctx_barrier", self.h)

    def device_info(self):
        """{"device": HIP ordinal, "pci_bus_id": "0000:..", "transport":
        "single" | "rccl" | "host" | "ipc"} of this rank."""
        dev, tr = C.c_int(), C.c_int()
        pci = C.create_string_buffer(32)
        call("kle_ctx_get_device", self.h, C.byref(dev), pci, 32, C.byref(tr))
        return {"device": dev.value, "pci_bus_id": pci.value.decode(),
                "transport": ("single", "rccl", "host", "ipc")[tr.value]}

    def comm_info(self):
        """(ranks, this rank) as the RCCL communicator reports them
        (ncclCommCount / ncclCommUserRank), or (0, -1) without one."""
        cnt, rk = C.c_int(), C.c_int()
        call("kle_ctx_get_comm_info", self.h, C.byref(cnt), C.byref(rk))
        return cnt.value, rk.value

    def set_profiling(self, on=True, only=None, every=1):
        """Event-time device launches; `only` restricts it to one kernel tag,
        `every` > 1 times one launch in `every` (sampled)."""
        call("kle_ctx_set_profiling_filter", self.h, only.encode() if only else None)
        call("kle_ctx_set_profiling_sample", self.h, int(every))
        call("kle_ctx_set_profiling", self.h, int(bool(on)))

    def kernel_stats(self, name):
        cnt, ms = C.c_int64(), C.c_double()
        call("kle_ctx_get_kernel_stats", self.h, name.encode(), C.byref(cnt), C.byref(ms))
        return cnt.value, ms.value

    def reset_stats(self):
        call("kle_ctx_reset_kernel_stats", self.h)

    def stream_copy_gbps(self, nbytes=1 << 30, reps=20):
        g = C.c_double()
        call("kle_stream_bench", self.h, int(nbytes), int(reps), 0, C.byref(g))
        return g.value

    def stream_read_gbps(self, nbytes=1 << 31, reps=20):
        g = C.c_double()
        call("kle_stream_bench", self.h, int(nbytes), int(reps), 1, C.byref(g))
        return g.value

    def destroy(self):
        if self.h:
            call("kle_ctx_destroy", self.h)
            self.h = None


_CTX = None


def get_ctx():
    global _CTX
    if _CTX is None:
        if os.environ.get("KLE_NB_PAD"):
            set_row_padding(int(os.environ["KLE_NB_PAD"]))
        if os.environ.get("KLE_NB_LAYOUT"):
            set_value_layout(int(os.environ["KLE_NB_LAYOUT"]))
        if os.environ.get("KLE_SPMV_WAVES"):
            set_tuning("spmv_waves", int(os.environ["KLE_SPMV_WAVES"]))
        if os.environ.get("KLE_SPMV_SYM"):
            set_tuning("spmv_sym", int(os.environ["KLE_SPMV_SYM"]))
        if os.environ.get("KLE_SPMV_SYM_MIN_ROWS"):
            set_tuning("spmv_sym_min_rows", int(os.environ["KLE_SPMV_SYM_MIN_ROWS"]))
        if os.environ.get("KLE_SPMV_DICT_MIN_ROWS"):
            set_tuning("spmv_dict_min_rows", int(os.environ["KLE_SPMV_DICT_MIN_ROWS"]))
        if os.environ.get("KLE_SPMV_SYM_TILE64"):
            set_tuning("spmv_sym_tile64", int(os.environ["KLE_SPMV_SYM_TILE64"]))
        if os.environ.get("KLE_SPMV_SYM_BRICK"):
            set_tuning("spmv_sym_brick", int(os.environ["KLE_SPMV_SYM_BRICK"]))
        if os.environ.get("KLE_KSP_REFINE"):
            set_tuning("ksp_refine", int(os.environ["KLE_KSP_REFINE"]))
        if os.environ.get("KLE_SPMV_GSYM_BRICK"):
            set_tuning("spmv_gsym_brick", int(os.environ["KLE_SPMV_GSYM_BRICK"]))
        if os.environ.get("KLE_TUNING"):  # any knobs, as JSON: KLE_TUNING='{"spmv_gather_wps": 2}'
            import json
            for k, v in json.loads(os.environ["KLE_TUNING"]).items():
                set_tuning(k, int(v))
        _CTX = Context()
    return _CTX


def set_row_padding(quantum):
    """Row padding quantum (blocks) for node-block matrices created afterwards
    (KLE_NB_PAD in the environment sets the initial value)."""
    call("kle_set_nb_pad", int(quantum))


def set_value_layout(layout):
    """Node-block value layout for matrices created afterwards (0 padded
    streams, 1 chunked + packed tail); KLE_NB_LAYOUT sets the initial value."""
    call("kle_set_nb_layout", int(layout))


def set_tuning(key, value):
    """libkle performance knob (kle_set_tuning): "spmv_waves"; every setting
    gives correct results."""
    call("kle_set_tuning", key.encode(), int(value))


def get_tuning(key):
    v = C.c_int()
    call("kle_get_tuning", key.encode(), C.byref(v))
    return v.value


def get_value_layout():
    return int(load().kle_get_nb_layout())


def get_row_padding():
    return int(load().kle_get_nb_pad())


def set_ctx(ctx):
    global _CTX
    _CTX = ctx


def finalize():
    global _CTX
    if _CTX is not None:
        _CTX.destroy()
        _CTX = None
