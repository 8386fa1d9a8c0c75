"""Image-parallel sharding and the one collective of the codec: an all-gather of
per-rank rate / distortion statistics.

One process per GPU (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/
``MASTER_PORT`` from the launcher's environment).  Images are independent, so the
data path has no collective at all; at the end each rank contributes a 48-byte
``RankStats`` record and every rank computes the dataset PSNR exactly as
processing_utils/evaluate.py:10-32 does (sum of SSE over sum of dims), the bpp as
bytes*8/pixels (evaluate.py:45-50) and the throughput as total pixels over
(max end - min start).

Backends:
* ``RcclComm`` — RCCL (librccl.so, ctypes) over xGMI on the codec's HIP stream; the
  ncclUniqueId is bootstrapped through a tiny TCP exchange on MASTER_ADDR.  Used by
  bench.py / the CLIs on GPU boxes.  No PyTorch is imported in GPU processes (torch
  bundles a second HIP runtime with the same soname).
* ``GlooComm`` — torch.distributed gloo on CPU, for the world_size-2 CPU tests of the
  same orchestration code.
* ``LocalComm`` — world size 1.
"""
from __future__ import annotations

import ctypes as C
import os
import socket
import struct
import sys
import threading
import time
from dataclasses import dataclass

import numpy as np

STATS_FIELDS = ("sse", "dims", "bits", "images", "t_start", "t_end")


@dataclass
class RankStats:
    sse: float = 0.0      # sum of squared errors over the rank's images (float64)
    dims: int = 0         # number of sample values (H*W*3 per image)
    bits: int = 0         # raw code bits (or coded bytes*8 once entropy coded)
    images: int = 0
    t_start: float = 0.0  # wall clock (time.time()) at the start of the rank's work
    t_end: float = 0.0

    def to_array(self) -> np.ndarray:
        return np.array([self.sse, self.dims, self.bits, self.images, self.t_start, self.t_end], np.float64)

    @staticmethod
    def from_array(a) -> "RankStats":
        a = np.asarray(a, np.float64)
        return RankStats(float(a[0]), int(a[1]), int(a[2]), int(a[3]), float(a[4]), float(a[5]))


def combine(stats: list[RankStats]) -> dict:
    """Global metrics from every rank's record (processing_utils/evaluate.py:10-32,45-50)."""
    sse = sum(s.sse for s in stats)
    dims = sum(s.dims for s in stats)
    bits = sum(s.bits for s in stats)
    pixels = dims / 3.0
    t0 = min(s.t_start for s in stats)
    t1 = max(s.t_end for s in stats)
    psnr = float("inf") if sse == 0 else 20.0 * np.log10(255.0) - 10.0 * np.log10(sse / max(dims, 1))
    return {
        "psnr_db": float(psnr),
        "bpp": bits / pixels if pixels else 0.0,
        "images": sum(s.images for s in stats),
        "pixels": int(pixels),
        "seconds": t1 - t0,
        "mpix_per_s": pixels / (t1 - t0) / 1e6 if t1 > t0 else float("nan"),
    }


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Static contiguous split [r*ceil(M/W), ...): rank r gets items [lo, hi)."""
    per = -(-n_items // world)
    lo = min(n_items, rank * per)
    return lo, min(n_items, lo + per)


def env_rank() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


# Bounds of the blocking waits (seconds).  Creating the communicator and the id rendezvous
# happen right after every rank starts, so a short bound catches a missing peer early
# (TIC_DIST_TIMEOUT).  A collective also waits for every peer to ARRIVE at it: a collective
# that follows rank-dependent work (a tuning run on some ranks, rank 0's CPU baseline, an
# uneven shard) gets a bound sized for that work — the caller passes
# timeout=collective_timeout() (TIC_DIST_COLLECTIVE_TIMEOUT) — and every other collective
# (the per-step ones: ranks arrive after the same work) keeps a short default bound,
# step_timeout() (TIC_DIST_STEP_TIMEOUT, default the init bound), so a peer that dies in the
# steady state ends the job in minutes, not half an hour.
INIT_TIMEOUT = 150.0
COLLECTIVE_TIMEOUT = 1800.0


def init_timeout() -> float:
    return float(os.environ.get("TIC_DIST_TIMEOUT", INIT_TIMEOUT))


def collective_timeout() -> float:
    """The bound of a collective that follows rank-dependent work (pass it explicitly)."""
    return float(os.environ.get("TIC_DIST_COLLECTIVE_TIMEOUT", COLLECTIVE_TIMEOUT))


def step_timeout() -> float:
    """The default bound of every other collective."""
    return float(os.environ.get("TIC_DIST_STEP_TIMEOUT", init_timeout()))


class Deadline:
    """A bounded wait around a blocking call that can hang when a peer never arrives (RCCL
    communicator creation, a collective and its synchronisation, the id rendezvous): if the
    call has not returned after `seconds`, say which rank waited for what and end the process
    with exit code 3 — a clear failure instead of a stalled multi-GPU run (never a re-exec;
    the GPU is released by the process exit).  An explicit `seconds` is used as given; with
    None the init bound applies (init_timeout(): TIC_DIST_TIMEOUT or 150 s)."""

    def __init__(self, what: str, seconds: float | None = None, rank: int | None = None):
        self.what = what
        self.seconds = float(seconds) if seconds is not None else init_timeout()
        self.rank = env_rank()[0] if rank is None else rank
        self._timer = None

    def _fire(self):
        sys.stderr.write(f"[rank {self.rank}] {self.what} did not complete within {self.seconds:.0f} s "
                         f"(a peer rank is missing or stalled): exiting with code 3\n")
        sys.stderr.flush()
        os._exit(3)

    def __enter__(self):
        self._timer = threading.Timer(self.seconds, self._fire)
        self._timer.daemon = True
        self._timer.start()
        return self

    def __exit__(self, *exc):
        self._timer.cancel()
        return False


class LocalComm:
    rank, world = 0, 1

    def barrier(self, timeout: float | None = None):
        pass

    def allreduce_max(self, x: float, timeout: float | None = None) -> float:
        return float(x)

    def allgather_stats(self, s: RankStats, timeout: float | None = None) -> list[RankStats]:
        return [s]

    def allgather_f64(self, a, timeout: float | None = None) -> np.ndarray:
        return np.asarray(a, np.float64).reshape(1, -1)

    def close(self):
        pass


class GlooComm:
    """torch.distributed (gloo, CPU) — for CPU tests of the multi-rank path only; its waits
    carry the same bounds as RcclComm's."""

    def __init__(self):
        import torch.distributed as dist  # imported lazily: never in GPU processes
        self.dist = dist
        if not dist.is_initialized():
            with Deadline("gloo init_process_group", init_timeout()):
                dist.init_process_group("gloo")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def _bound(self, what, timeout):
        return Deadline(what, step_timeout() if timeout is None else timeout, self.rank)

    def barrier(self, timeout: float | None = None):
        with self._bound("gloo barrier", timeout):
            self.dist.barrier()

    def allreduce_max(self, x: float, timeout: float | None = None) -> float:
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        with self._bound("gloo all_reduce(max)", timeout):
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def allgather_stats(self, s: RankStats, timeout: float | None = None) -> list[RankStats]:
        return [RankStats.from_array(r) for r in self.allgather_f64(s.to_array(), timeout)]

    def allgather_f64(self, a, timeout: float | None = None) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a, np.float64).reshape(-1))
        out = [torch.zeros_like(t) for _ in range(self.world)]
        with self._bound("gloo all_gather", timeout):
            self.dist.all_gather(out, t)
        return np.stack([o.numpy() for o in out])

    def close(self):
        self.dist.destroy_process_group()


# ----------------------------------------------------------------------------- RCCL
NCCL_FLOAT64 = 8
NCCL_MAX = 2
NCCL_UNIQUE_ID_BYTES = 128


class _NcclUniqueId(C.Structure):
    # c_ubyte, not c_char: a c_char array field reads back as bytes cut at the first NUL,
    # and the id (a sockaddr + magic) is full of zero bytes
    _fields_ = [("internal", C.c_ubyte * NCCL_UNIQUE_ID_BYTES)]


def uid_to_bytes(uid: _NcclUniqueId) -> bytes:
    """All 128 bytes of an ncclUniqueId."""
    return C.string_at(C.addressof(uid), NCCL_UNIQUE_ID_BYTES)


def uid_from_bytes(raw: bytes) -> _NcclUniqueId:
    if len(raw) != NCCL_UNIQUE_ID_BYTES:
        raise ValueError(f"ncclUniqueId must be {NCCL_UNIQUE_ID_BYTES} bytes, got {len(raw)}")
    uid = _NcclUniqueId()
    C.memmove(C.addressof(uid), raw, NCCL_UNIQUE_ID_BYTES)
    return uid


def _recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed")
        buf += chunk
    return buf


def exchange_unique_id(rank: int, world: int, payload: bytes | None, addr: str, port: int,
                       timeout: float = 120.0) -> bytes:
    """Rank 0 serves `payload` (the 128-byte ncclUniqueId) to world-1 peers over TCP."""
    if world == 1:
        return payload
    if rank == 0:
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((addr, port))
        srv.listen(world)
        srv.settimeout(timeout)
        try:
            for _ in range(world - 1):
                conn, _ = srv.accept()
                with conn:
                    conn.sendall(struct.pack("!I", len(payload)) + payload)
        finally:
            srv.close()
        return payload
    deadline = time.time() + timeout
    while True:
        try:
            with socket.create_connection((addr, port), timeout=5.0) as s:
                (ln,) = struct.unpack("!I", _recv_exact(s, 4))
                return _recv_exact(s, ln)
        except (ConnectionRefusedError, socket.timeout, OSError):
            if time.time() > deadline:
                raise
            time.sleep(0.05)


class RcclComm:
    """RCCL communicator over the codec's HIP stream (ctypes; no PyTorch)."""

    def __init__(self, codec, rank: int, world: int, addr: str | None = None, port: int | None = None):
        self.rank, self.world, self.codec = rank, world, codec
        self.nccl = C.CDLL(os.environ.get("TIC_RCCL", "/opt/rocm/lib/librccl.so.1"))
        self.nccl.ncclGetUniqueId.argtypes = [C.POINTER(_NcclUniqueId)]
        self.nccl.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _NcclUniqueId, C.c_int]
        self.nccl.ncclAllGather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p]
        self.nccl.ncclAllReduce.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p]
        self.nccl.ncclGetErrorString.restype = C.c_char_p
        self.nccl.ncclCommDestroy.argtypes = [C.c_void_p]
        uid = _NcclUniqueId()
        if rank == 0:
            self._ok(self.nccl.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = port or int(os.environ.get("TIC_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 17))
        with Deadline(f"ncclUniqueId rendezvous on {addr}:{port}", init_timeout(), rank):
            raw = exchange_unique_id(rank, world, uid_to_bytes(uid) if rank == 0 else None, addr, port)
        uid = uid_from_bytes(raw)
        self.comm = C.c_void_p()
        with Deadline(f"ncclCommInitRank (world {world})", init_timeout(), rank):
            self._ok(self.nccl.ncclCommInitRank(C.byref(self.comm), world, uid, rank), "ncclCommInitRank")
        self.stream = codec.stream_ptr()
        # every collective below is followed by a synchronisation, so nothing of ours stays
        # pending on the codec's stream: its lanes need not fork from it at every call
        codec.stream_external(False)
        self.cap = 16  # f64 words per rank a gather carries
        self.d_send = codec.alloc(8 * self.cap)
        self.d_recv = codec.alloc(8 * self.cap * world)

    def _ok(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.nccl.ncclGetErrorString(rc).decode()} ({rc})")

    def allreduce_max(self, x: float, timeout: float | None = None) -> float:
        self.d_send.upload(np.array([x], np.float64))
        with Deadline("ncclAllReduce(max)", step_timeout() if timeout is None else timeout, self.rank):
            self._ok(self.nccl.ncclAllReduce(self.d_send.ptr, self.d_recv.ptr, 1, NCCL_FLOAT64, NCCL_MAX, self.comm,
                                             self.stream), "ncclAllReduce")
            self.codec.synchronize()
        return float(self.d_recv.download((1,), np.float64)[0])

    def barrier(self, timeout: float | None = None):
        self.allreduce_max(0.0, timeout)

    def allgather_f64(self, a, timeout: float | None = None) -> np.ndarray:
        """[world, k] f64: every rank's k words (k <= 16), one ncclAllGather on the codec stream."""
        a = np.ascontiguousarray(a, np.float64).reshape(-1)
        if a.size > self.cap:
            raise ValueError(f"allgather_f64 carries at most {self.cap} words per rank")
        self.d_send.upload(a)
        with Deadline("ncclAllGather", step_timeout() if timeout is None else timeout, self.rank):
            self._ok(self.nccl.ncclAllGather(self.d_send.ptr, self.d_recv.ptr, a.size, NCCL_FLOAT64, self.comm,
                                             self.stream), "ncclAllGather")
            self.codec.synchronize()
        return self.d_recv.download((self.world, a.size), np.float64)

    def allgather_stats(self, s: RankStats, timeout: float | None = None) -> list[RankStats]:
        return [RankStats.from_array(r) for r in self.allgather_f64(s.to_array(), timeout)]

    def close(self):
        if self.comm:
            self.nccl.ncclCommDestroy(self.comm)
            self.comm = None


def make_comm(codec=None):
    """LocalComm at world size 1, RcclComm on a GPU codec otherwise.  Every rank passes one
    barrier here, under the short init bound, before any rank-dependent work: a missing peer
    is reported at start-up, and the later collectives only wait for work, never for a rank
    that is not there."""
    rank, world, _ = env_rank()
    if world == 1:
        return LocalComm()
    comm = GlooComm() if codec is None else RcclComm(codec, rank, world)
    comm.barrier(init_timeout())
    return comm


def all_ranks(comm, flag: bool, timeout: float | None = None) -> bool:
    """True on every rank iff `flag` is true on every rank (one max-reduce of the negation):
    a decision every rank must take alike (e.g. whether to run the minutes-long tuning
    before the first barrier) is taken from all ranks' inputs.  Ranks reach it after
    rank-dependent work, so its bound is the collective one unless given."""
    return comm.allreduce_max(0.0 if flag else 1.0, collective_timeout() if timeout is None else timeout) == 0.0
