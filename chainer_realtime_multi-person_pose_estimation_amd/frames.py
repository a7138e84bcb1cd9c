"""Frame-parallel serving across GPUs (one process per GPU, no PyTorch).

``PoseDetector.__call__`` (pose_detector.py:484-517) keeps no cross-frame state, so a stream of
frames shards with no data-path collective: frame i goes to rank i % world, and each rank runs its
frames on its own device-resident replica.  The only exchange is a gather of fixed-size per-frame
result records to rank 0 (include/openpose_hip.h "Multi-GPU result gather"):

* ``RcclGather`` -- the product path: records packed on the device after the post-process and
  gathered by ``ncclGather`` straight from HBM on a communicator stream (gather.hip), double
  buffered so step k's gather overlaps step k+1's compute, with a per-rank timeout.
* ``HostGather`` -- the same records and control flow over TCP sockets from host memory (CPU
  tests, world size 2, and any rank without a GPU).

``SocketTransport`` is the small TCP star (rank 0 = hub) both use for bootstrap (RCCL's unique id),
barriers and scalar max-reductions; every receive has a timeout, so a stalled rank fails loudly
(``TimeoutError``) instead of hanging the job (SURVEY §5 failure detection).
"""
import os
import socket
import struct
import time

import numpy as np

N_JOINTS = 18
STATUS_CAPACITY = 3  # OP_ERR_CAPACITY (include/openpose_hip.h): the frame exceeded the batched caps
HDR_BYTES = 32  # int32 status, n_peaks, n_persons, 0; int64 frame id; 8 pad


def shard(n_frames, rank, world):
    """Frame ids owned by `rank` (round-robin)."""
    return list(range(rank, n_frames, world))


def record_bytes(max_persons):
    return HDR_BYTES + max_persons * (N_JOINTS * 3 + 1) * 8


def pack_records(results, max_persons):
    """Host-side records, byte-identical to the device's pack_records (runtime.hip).
    results: [(frame_id, status, n_peaks, poses (P,18,3), scores (P,))] -> (n, record_bytes) uint8."""
    rb = record_bytes(max_persons)
    out = np.zeros((len(results), rb), np.uint8)
    for i, (fid, status, n_peaks, poses, scores) in enumerate(results):
        n_persons = len(scores) if status == 0 else 0
        k = min(n_persons, max_persons)
        hdr = np.frombuffer(struct.pack("<iiiiqq", int(status), int(n_peaks), int(n_persons), 0, int(fid), 0), np.uint8)
        out[i, :HDR_BYTES] = hdr
        body = np.zeros(max_persons * (N_JOINTS * 3 + 1), np.float64)
        body[:k * N_JOINTS * 3] = np.asarray(poses, np.float64)[:k].reshape(-1)
        body[max_persons * N_JOINTS * 3:max_persons * N_JOINTS * 3 + k] = np.asarray(scores, np.float64)[:k]
        out[i, HDR_BYTES:] = body.view(np.uint8)
    return out


def unpack_records(buf, max_persons):
    """(n, record_bytes) uint8 (or raw bytes) -> [(frame_id, status, n_peaks, poses, scores)] in
    frame-id order; frames carry at most max_persons persons (status/n_peaks always exact)."""
    rb = record_bytes(max_persons)
    a = np.frombuffer(buf, np.uint8).reshape(-1, rb) if not isinstance(buf, np.ndarray) else buf.reshape(-1, rb)
    out = []
    for row in a:
        status, n_peaks, n_persons, _, fid, _ = struct.unpack("<iiiiqq", row[:HDR_BYTES].tobytes())
        body = row[HDR_BYTES:].view(np.float64)
        k = min(n_persons, max_persons)
        poses = body[:k * N_JOINTS * 3].reshape(k, N_JOINTS, 3).copy()
        scores = body[max_persons * N_JOINTS * 3:max_persons * N_JOINTS * 3 + k].copy()
        out.append((fid, status, n_peaks, poses, scores))
    out.sort(key=lambda r: r[0])
    return out


def count_persons(buf, max_persons):
    """(sum of the exact per-frame person counts, frames whose status is OP_ERR_CAPACITY = over
    the batched post-process caps, to be fetched with op_fetch_result) of packed records."""
    rb = record_bytes(max_persons)
    a = np.frombuffer(buf, np.uint8).reshape(-1, rb)
    hdr = np.ascontiguousarray(a[:, :HDR_BYTES]).view(np.int32)  # status, n_peaks, n_persons, ...
    ok = hdr[:, 0] == 0
    return int(hdr[ok, 2].sum()), int((hdr[:, 0] == STATUS_CAPACITY).sum())


# ---------------------------------------------------------------- transport
def _recv_exact(sock, n):
    chunks, got = [], 0
    while got < n:
        b = sock.recv(min(n - got, 1 << 20))
        if not b:
            raise ConnectionError("peer closed the connection")
        chunks.append(b)
        got += len(b)
    return b"".join(chunks)


def _send_msg(sock, payload):
    sock.sendall(struct.pack("<q", len(payload)) + payload)


def _recv_msg(sock):
    (n,) = struct.unpack("<q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class SocketTransport(object):
    """TCP star of `world` ranks on one node: rank 0 listens on (addr, port), every other rank
    connects.  All operations are collective and time out after `timeout` seconds."""

    def __init__(self, rank, world, addr="127.0.0.1", port=None, timeout=120.0):
        self.rank, self.world, self.timeout = int(rank), int(world), float(timeout)
        self.peers = {}
        if self.world == 1:
            return
        port = int(port if port is not None else default_port())
        deadline = time.monotonic() + self.timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(self.timeout)
            try:
                while len(self.peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(self.timeout)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    self.peers[r] = conn
            except socket.timeout:
                raise TimeoutError("rank 0: only %d of %d ranks connected within %.0f s"
                                   % (len(self.peers) + 1, self.world, self.timeout))
            finally:
                srv.close()
        else:
            while True:
                try:
                    conn = socket.create_connection((addr, port), timeout=max(0.1, deadline - time.monotonic()))
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise TimeoutError("rank %d: rank 0 not reachable at %s:%d within %.0f s"
                                           % (self.rank, addr, port, self.timeout))
                    time.sleep(0.05)
            conn.settimeout(self.timeout)
            conn.sendall(struct.pack("<i", self.rank))
            self.peers[0] = conn

    def _io(self, fn, what):
        try:
            return fn()
        except socket.timeout:
            raise TimeoutError("rank %d: %s timed out after %.0f s (a rank stalled or died)"
                               % (self.rank, what, self.timeout))

    def gather(self, payload):
        """Rank 0: [payload of rank 0, 1, ...]; other ranks: None."""
        if self.world == 1:
            return [payload]
        if self.rank != 0:
            self._io(lambda: _send_msg(self.peers[0], payload), "gather")
            return None
        return [payload] + [self._io(lambda r=r: _recv_msg(self.peers[r]), "gather from rank %d" % r)
                            for r in range(1, self.world)]

    def broadcast(self, payload=None):
        """Rank 0's payload on every rank."""
        if self.world == 1:
            return payload
        if self.rank == 0:
            for r in range(1, self.world):
                self._io(lambda r=r: _send_msg(self.peers[r], payload), "broadcast")
            return payload
        return self._io(lambda: _recv_msg(self.peers[0]), "broadcast")

    def barrier(self):
        self.gather(b"")
        self.broadcast(b"" if self.rank == 0 else None)

    def all_reduce(self, value, op="max"):
        """max / sum of one float over ranks, on every rank."""
        got = self.gather(struct.pack("<d", float(value)))
        res = None
        if got is not None:
            vals = [struct.unpack("<d", g)[0] for g in got]
            res = struct.pack("<d", max(vals) if op == "max" else sum(vals))
        return struct.unpack("<d", self.broadcast(res))[0]

    def close(self):
        for c in self.peers.values():
            try:
                c.close()
            except OSError:
                pass
        self.peers = {}


def default_port():
    """Port of the transport's hub: OP_STORE_PORT, else MASTER_PORT + 101 (torchrun's own store
    holds MASTER_PORT), else 29611."""
    if os.environ.get("OP_STORE_PORT"):
        return int(os.environ["OP_STORE_PORT"])
    if os.environ.get("MASTER_PORT"):
        return (int(os.environ["MASTER_PORT"]) + 101) % 65536
    return 29611


# ---------------------------------------------------------------- gathers
class HostGather(object):
    """Result records gathered over the socket transport from host memory (CPU path)."""

    def __init__(self, transport, max_persons=64):
        self.t, self.max_persons = transport, int(max_persons)
        self.pending = []

    def submit(self, results):
        """results: this rank's [(frame_id, status, n_peaks, poses, scores)] of one step."""
        self.pending.append(pack_records(results, self.max_persons).tobytes())

    def wait(self, timeout=None):
        """Rank 0: every rank's records of the oldest submitted step, by frame id; else None."""
        got = self.t.gather(self.pending.pop(0))
        if got is None:
            return None
        return unpack_records(b"".join(got), self.max_persons)


class RcclGather(object):
    """Result records packed on the device and gathered to rank 0 by RCCL (gather.hip)."""

    def __init__(self, ctx, transport, max_persons=64, timeout=120.0):
        import ctypes
        from . import _lib
        self._lib, self._ct = _lib, ctypes
        self.ctx, self.t, self.max_persons, self.timeout = ctx, transport, int(max_persons), float(timeout)
        L = _lib.lib()
        uid = (ctypes.c_uint8 * _lib.OP_COMM_ID_BYTES)()
        if transport.rank == 0:
            _lib.check(L.op_comm_unique_id(uid), "op_comm_unique_id")
        raw = transport.broadcast(bytes(uid) if transport.rank == 0 else None)
        uid = (ctypes.c_uint8 * _lib.OP_COMM_ID_BYTES).from_buffer_copy(raw)
        h = ctypes.c_void_p()
        _lib.check(L.op_comm_create(ctx.h, transport.world, transport.rank, uid, self.timeout, ctypes.byref(h)),
                   "op_comm_create")
        self.h = h

    def submit(self, first, n, frame_base, frame_stride):
        """Enqueue the gather of this rank's staged frames [first, first+n) (global ids
        frame_base + i * frame_stride) behind the context's queued work; returns at once."""
        self._lib.check(self._lib.lib().op_comm_gather_results(self.h, self.ctx.h, int(first), int(n),
                                                               self.max_persons, int(frame_base),
                                                               int(frame_stride)), "op_comm_gather_results")

    def wait(self, timeout=None, raw=False):
        """Rank 0: every rank's records of the oldest submitted step (unpacked, by frame id; or the
        raw record bytes with raw=True); other ranks: None."""
        ct = self._ct
        p, nf, rb = ct.c_void_p(), ct.c_int32(), ct.c_int64()
        self._lib.check(self._lib.lib().op_comm_wait(self.h, float(timeout or self.timeout), ct.byref(p),
                                                     ct.byref(nf), ct.byref(rb)), "op_comm_wait")
        if not p.value:
            return None
        buf = ct.string_at(p.value, nf.value * rb.value)
        return buf if raw else unpack_records(buf, self.max_persons)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._lib.lib().op_comm_destroy(self.h)
            self.h = None
