"""Host-side orchestration of the walker-sharded multi-GPU run.

One process per GPU.  Walkers are independent, so rank r owns a contiguous range of
global walker indices and seeds walker w with ``base + w``: the chains do not depend
on the GPU count.  Ranks talk only through the host group (barrier, timing max, the
128-byte RCCL id) and, at the end, through RCCL in libolpe (all-gather of states and
chains, all-reduce of moments).  The reference's equivalent is mpi4py's
``comm.barrier()`` once per iteration (apf_step2.py:338), which carries no data.

The host group is plain TCP from the standard library (no PyTorch): a star around
rank 0 on ``MASTER_ADDR``.  torchrun (``python -m torch.distributed.run``) keeps
working as the launcher -- it only supplies RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT -- but its agent already listens on MASTER_PORT, so the group
listens on the first free port of MASTER_PORT+1 .. MASTER_PORT+32 (or
``OLPE_HOST_PORT``) and the other ranks find it by a handshake token (job port, world
size, torchrun run id) on that range.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

import numpy as np

PORT_SPAN = 32


def env():
    """(rank, world_size, local_rank) from the torchrun / mpirun-style environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def rank_device(local: int, visible: int) -> int:
    """HIP device of the rank with LOCAL_RANK ``local`` when the process sees ``visible``
    devices: its own ordinal when every GPU is visible (torchrun, bench.py --gpus), 0
    when the launcher gave each process one GPU (HIP_VISIBLE_DEVICES per rank).  Whether
    the ranks then hold distinct GPUs is checked by PCI bus id (bench.py)."""
    if visible <= 0 or local < visible:
        return local
    if visible == 1:
        return 0
    raise ValueError(f"LOCAL_RANK {local} but this process sees {visible} GPUs")


def node_id() -> str:
    """This machine's identity for telling GPUs apart across nodes: the kernel's boot id
    (unique per boot of a host, the same for every process on it), else the host name.
    PCI bus ids alone repeat across identical nodes (0000:05:00.0 on each of them).
    ``OLPE_NODE_ID`` overrides it (the CPU tests' fake nodes)."""
    if os.environ.get("OLPE_NODE_ID"):
        return os.environ["OLPE_NODE_ID"]
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            bid = f.read().strip()
            if bid:
                return bid
    except OSError:
        pass
    return socket.gethostname()


def shared_gpus(placement) -> list:
    """The (node, PCI bus id) pairs that more than one rank holds, from every rank's
    ``(node_id(), pci_id)`` in rank order (the same list on every rank after an
    allgather, so every rank reaches the same verdict).  Empty when every rank has a GPU
    of its own; ranks on different nodes may report the same bus id."""
    seen, dup = set(), []
    for p in placement:
        key = (p[0], p[1])
        if key in seen and key not in dup:
            dup.append(key)
        seen.add(key)
    return dup


def shard(total: int, world: int, rank: int):
    """Contiguous shard [w0, w0 + n) of ``total`` walkers for ``rank`` (strong split;
    shard sizes differ by at most one, so the RCCL gathers, which need equal counts,
    are only used with ``total % world == 0`` -- libolpe checks)."""
    lo = (rank * total) // world
    hi = ((rank + 1) * total) // world
    return lo, hi - lo


def walker_seeds(base: int, w0: int, n: int) -> np.ndarray:
    """np.random.seed values of walkers w0 .. w0+n-1 (global index -> seed)."""
    return ((int(base) + w0 + np.arange(n, dtype=np.int64)) & 0xFFFFFFFF).astype(np.uint32)


# ----------------------------------------------------------------------------------
# length-prefixed messages
# ----------------------------------------------------------------------------------
def _send(sock, payload: bytes):
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("host group peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


def _pack(obj) -> bytes:
    if isinstance(obj, (bytes, bytearray)):
        return b"b" + bytes(obj)
    return b"j" + json.dumps(obj).encode()


def _unpack(b: bytes):
    return b[1:] if b[:1] == b"b" else json.loads(b[1:].decode())


class HostGroup:
    """Barrier / max / sum / broadcast over a TCP star; a no-op group when world == 1."""

    def __init__(self, rank: int, world: int, timeout_s: float = 600.0,
                 addr: str | None = None, port: int | None = None):
        self.rank, self.world = rank, world
        self.conns = {}          # rank 0: peer rank -> socket
        self.sock = None         # rank > 0: the connection to rank 0
        self.server = None
        if world <= 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("OLPE_HOST_PORT",
                                      int(os.environ.get("MASTER_PORT", "29500")) + 1))
        token = "olpe-hostgroup:%s:%d:%s" % (os.environ.get("MASTER_PORT", ""), world,
                                             os.environ.get("TORCHELASTIC_RUN_ID", ""))
        deadline = time.monotonic() + timeout_s
        if rank == 0:
            self._serve(addr, port, token, deadline)
        else:
            self._join(addr, port, token, deadline)

    # -- rendezvous ----------------------------------------------------------------
    def _serve(self, addr, port, token, deadline):
        err = None
        for p in range(port, port + PORT_SPAN):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                s.bind((addr, p))
            except OSError as e:
                s.close()
                err = e
                continue
            s.listen(max(16, self.world))
            self.server = s
            break
        if self.server is None:
            raise OSError(f"host group: no free port in {port}..{port + PORT_SPAN - 1}: {err}")
        while len(self.conns) < self.world - 1:
            self.server.settimeout(max(0.1, deadline - time.monotonic()))
            try:
                c, _ = self.server.accept()
            except socket.timeout:
                raise TimeoutError(f"host group: {len(self.conns) + 1} of {self.world} ranks "
                                   "joined before the timeout") from None
            c.settimeout(10.0)
            try:
                hello = json.loads(_recv(c).decode())
            except (OSError, ValueError, ConnectionError):
                c.close()
                continue
            if hello.get("token") != token or not 0 < int(hello.get("rank", -1)) < self.world \
                    or int(hello["rank"]) in self.conns:
                c.close()                    # someone else's job on this port range
                continue
            _send(c, json.dumps({"token": token}).encode())
            c.settimeout(None)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.conns[int(hello["rank"])] = c

    def _join(self, addr, port, token, deadline):
        hello = json.dumps({"token": token, "rank": self.rank}).encode()
        while time.monotonic() < deadline:
            for p in range(port, port + PORT_SPAN):
                try:
                    c = socket.create_connection((addr, p), timeout=2.0)
                except OSError:
                    continue
                try:
                    _send(c, hello)
                    ack = json.loads(_recv(c).decode())
                except (OSError, ValueError, ConnectionError):
                    c.close()
                    continue
                if ack.get("token") != token:
                    c.close()
                    continue
                c.settimeout(None)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self.sock = c
                return
            time.sleep(0.2)
        raise TimeoutError(f"host group: rank {self.rank} found no rank 0 on "
                           f"{addr}:{port}..{port + PORT_SPAN - 1}")

    # -- collectives ---------------------------------------------------------------
    def _gather(self, obj):
        """Root: list of every rank's obj (rank order); others: None."""
        if self.world <= 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [None] * (self.world - 1)
            for r, c in self.conns.items():
                out[r] = _unpack(_recv(c))
            return out
        _send(self.sock, _pack(obj))
        return None

    def broadcast(self, obj, src: int = 0):
        if self.world <= 1:
            return obj
        if src != 0:
            vals = self._gather(obj if self.rank == src else None)
            obj = vals[src] if self.rank == 0 else None
        if self.rank == 0:
            b = _pack(obj)
            for c in self.conns.values():
                _send(c, b)
            return obj
        return _unpack(_recv(self.sock))

    def barrier(self):
        self._gather(0)
        self.broadcast(0)

    def allmax(self, x: float) -> float:
        vals = self._gather(float(x))
        return float(self.broadcast(max(vals) if self.rank == 0 else None))

    def allsum(self, x: float) -> float:
        vals = self._gather(float(x))
        return float(self.broadcast(sum(vals) if self.rank == 0 else None))

    def allgather(self, obj):
        """Every rank's JSON-able obj, in rank order, on every rank."""
        return self.broadcast(self._gather(obj))

    def close(self):
        for c in list(self.conns.values()) + [self.sock, self.server]:
            if c is not None:
                try:
                    c.close()
                except OSError:
                    pass
        self.conns, self.sock, self.server = {}, None, None
