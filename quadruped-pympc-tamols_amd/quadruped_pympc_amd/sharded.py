"""Row-sharded sampling MPC over several GPUs (one process per GPU).

The reference runs all N rollouts of one MPC problem on one device
(centroidal_nmpc_jax.py:820-842: vmap over `num_parallel_computations`).  Here the rows of
one problem are split over ranks, rows [r*N/W, (r+1)*N/W) on rank r.  The only data exchange
of the step is one all-gather of a fixed-size per-rank record (rank order):

    [m_r, s_r, best row, pad | v_r (P) | K (row, cost) keys | K elite rows (K x P)]

with m_r the rank's minimum cost, s_r = sum exp(-(c - m_r)), v_r = sum exp(-(c - m_r)) * noise
(K = 1 except CEM, K = num_elite).  Every rank then merges the W records identically
(srbd_step_finish), so the new parameters agree bit for bit on all ranks without a broadcast.
Over RCCL the gather is `all_gather_into_tensor` on the stream the library launches on.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class RecordExchange:
    """The path's one collective: all-gather of equal-size float32 records in rank order."""

    def __init__(self, record_floats: int, world: int, device, group=None, stream=None):
        import torch

        self.torch = torch
        self.world = world
        self.group = group
        self.stream = stream  # the stream the record producer and the merge run on (CUDA only)
        self.local = torch.zeros(record_floats, dtype=torch.float32, device=device)
        self.gathered = torch.zeros(world * record_floats, dtype=torch.float32, device=device)
        self._parts = list(self.gathered.view(world, record_floats).unbind(0))

    def __call__(self) -> "torch.Tensor":
        import torch.distributed as dist

        if self.local.is_cuda:
            with self.torch.cuda.stream(self.stream):
                dist.all_gather_into_tensor(self.gathered, self.local, group=self.group)
        else:  # gloo: list form, written straight into the views of `gathered`
            dist.all_gather(self._parts, self.local, group=self.group)
        return self.gathered


def shard_rows(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(first row, row count) of `rank`: whole nodes of the reduction tree (srbd_shard_rows)."""
    return _lib.shard_rows(n_total, rank, world)


def torch_rccl_path() -> str:
    """The RCCL copy this process's torch already uses (dlopen of that path returns the same object)."""
    import os

    import torch

    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else ""


class ShardedSamplingMPC:
    """One rank of a row-sharded MPC problem on the current process's GPU.

    cfg: an _lib.SrbdConfig with the GLOBAL num_samples; rank / world_size / device_id are set here.

    transport="auto" (default): "xgmi" when its setup probe passes on every rank, else "rccl".
    transport="xgmi": the merge kernel stores its rank record straight into every rank's mailbox
    (IPC-mapped over xGMI) and merges the W records in the same launch: no collective launch, one
    merge kernel per step.  The IPC handles travel once over the torch process group.
    transport="rccl": the library owns an RCCL communicator (rank 0's ncclUniqueId is broadcast over
    the torch process group once) and runs rollout -> ncclAllGather -> merge from C++ on its own
    stream, so no Python sits between the kernels and the collective.
    rng: the device noise stream ('philox', or 'jax' / 'jax_legacy': the reference's jax.random stream keyed
    by the packed key, _lib.pack_key; draws are indexed by global row, so they are the same for any W).
    transport="torch": the record goes through torch.distributed.all_gather_into_tensor on a
    dedicated torch stream shared with the library (the legacy null stream cannot be handed to
    srbd_set_stream: a NULL handle selects the context's own stream).  Measured on one GPU: this
    Python-driven loop costs ~40-47 us per step against ~32 us for "rccl".
    """

    def __init__(self, cfg: _lib.SrbdConfig, rank: int, world: int, device_index: int, group=None,
                 transport: str = "auto", rng: str = "philox"):
        import torch

        cfg.rank, cfg.world_size, cfg.device_id = int(rank), int(world), int(device_index)
        cfg.use_graph = 0
        self.ctx = _lib.Context(cfg)
        if rng != "philox":  # the reference's jax.random stream: `seed` of step() is the packed key
            self.ctx.set_rng(rng)
        self.rank, self.world = rank, world
        self.device = torch.device("cuda", device_index)
        self.P = self.ctx.P
        self.result = _lib.SrbdResult()
        self.group = group
        if transport == "auto":
            transport = "xgmi" if self._setup_xgmi() else "rccl"
        elif transport == "xgmi":
            if not self._setup_xgmi():
                raise RuntimeError("xGMI exchange setup failed on at least one rank")
        if transport == "rccl":
            self._setup_rccl()
        elif transport == "torch":
            self.stream = torch.cuda.Stream(self.device)
            self.ctx.set_stream(self.stream.cuda_stream)
            with torch.cuda.stream(self.stream):
                self.exchange = RecordExchange(self.ctx.record_floats(), world, self.device, group, self.stream)
        elif transport != "xgmi":
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport

    def _setup_rccl(self):
        import torch.distributed as dist

        path = torch_rccl_path().encode()
        uid = (C.c_uint8 * 128)()
        if self.rank == 0:
            self.ctx.check(_lib.lib.srbd_comm_get_unique_id(path, uid), "srbd_comm_get_unique_id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        uid = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        self.ctx.check(_lib.lib.srbd_comm_init(self.ctx.h, path, uid), "srbd_comm_init")

    def _setup_xgmi(self) -> bool:
        """Export / exchange / connect / probe; True only when every rank succeeded."""
        import torch
        import torch.distributed as dist

        ok = 1
        handle = (C.c_uint8 * 64)()
        if _lib.lib.srbd_xgmi_export(self.ctx.h, handle) != _lib.OK:
            ok = 0
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle) if ok else b"", group=self.group)
        if ok and all(len(h) == 64 for h in handles):
            buf = (C.c_uint8 * (64 * self.world)).from_buffer_copy(b"".join(handles))
            if _lib.lib.srbd_xgmi_connect(self.ctx.h, buf) != _lib.OK:
                ok = 0
        else:
            ok = 0
        # every rank takes part in the probe (its wait is bounded), or none does
        flag = torch.tensor([ok], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            res = C.c_int32(0)
            if _lib.lib.srbd_xgmi_probe(self.ctx.h, C.byref(res)) != _lib.OK or res.value != 1:
                ok = 0
            flag = torch.tensor([ok], dtype=torch.int32, device=self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) != 1:
            _lib.lib.srbd_xgmi_disconnect(self.ctx.h)
            return False
        return True

    def step(self, state, ref, contact, best, sigma=None, noise_local=None, seed=42, counter=0):
        """One MPC iteration; returns (best, sigma, result) identical on every rank."""
        if self.transport in ("rccl", "xgmi"):
            b, sg, res, _ = self.ctx.step_sharded(state, ref, contact, best, sigma=sigma, noise_local=noise_local,
                                                  seed=seed, counter=counter)
            return b, sg, res
        f = lambda a: None if a is None else _lib.fptr(np.ascontiguousarray(a, np.float32))  # noqa: E731
        state = np.ascontiguousarray(state, np.float32)
        ref = np.ascontiguousarray(ref, np.float32)
        contact = np.ascontiguousarray(contact, np.float32)
        best = np.array(best, np.float32).reshape(self.P).copy()
        sig = None if sigma is None else np.array(np.broadcast_to(sigma, (self.P,)), np.float32)
        noise = None if noise_local is None else np.ascontiguousarray(noise_local, np.float32)
        h = self.ctx.h
        self.ctx.check(_lib.lib.srbd_step_local(h, f(state), f(ref), f(contact), contact.shape[1], f(best), f(sig),
                                                f(noise), C.c_uint64(int(seed)), C.c_uint64(int(counter)),
                                                C.c_void_p(self.exchange.local.data_ptr())), "srbd_step_local")
        g = self.exchange()
        self.ctx.check(_lib.lib.srbd_step_finish(h, C.c_void_p(g.data_ptr()), self.world, _lib.fptr(best), f(sig),
                                                 C.byref(self.result), None), "srbd_step_finish")
        return best, sig, self.result

    def device_steps(self, steps: int = 1) -> float:
        """`steps` device-resident steps (warm start kept on the device); returns elapsed ms."""
        if self.transport in ("rccl", "xgmi"):
            ms = C.c_float(0)
            self.ctx.check(_lib.lib.srbd_sharded_device_steps(self.ctx.h, int(steps), C.byref(ms)),
                           "srbd_sharded_device_steps")
            return float(ms.value)
        import torch

        h = self.ctx.h
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(self.stream)
        for _ in range(steps):
            self.ctx.check(_lib.lib.srbd_device_step_local(h, C.c_void_p(self.exchange.local.data_ptr())),
                           "srbd_device_step_local")
            g = self.exchange()
            self.ctx.check(_lib.lib.srbd_device_step_finish(h, C.c_void_p(g.data_ptr()), self.world),
                           "srbd_device_step_finish")
        ev1.record(self.stream)
        ev1.synchronize()
        return float(ev0.elapsed_time(ev1))

    def device_step(self):
        self.device_steps(1)

    def close(self):
        if self.transport == "torch":
            self.ctx.set_stream(None)
        self.ctx.close()
