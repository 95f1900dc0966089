"""Multi-GPU batch demodulation: one process per GPU, streams sharded, decoded
bytes all-gathered.  No torch: the control plane is a small
key-value store for the bootstrap and RCCL (libamr.so) for everything else.

Streams are independent, so a batch shards with no data-path exchange: rank r
demodulates the contiguous streams shard_range(B, r, world) on its own GPU.
The one collective is the all-gather of the decoded bytes (RCCL over xGMI),
after which every rank holds the whole batch's output, exactly as one
single-GPU call over the batch would have produced it.

Layers:
  * stores (the bootstrap: the RCCL unique id travels through one)
      FileStore   keys as files in a directory (the ranks of one node)
      TcpStore    keys in rank 0's memory, served over TCP (any ranks)
      store_from_env()   AMR_STORE=file:<dir> | tcp://<host>:<port>, else a
                  FileStore named after the launcher's MASTER_PORT and the
                  launcher process (torch.distributed.run starts the ranks
                  as children of one agent), so launch scripts need nothing new
  * transports: rank, world, all_gather(ndarray) -> [world, ...], max(),
    barrier()
      RcclTransport   RCCL through libamr.so (amr_comm_*): the product path;
                      also hands its communicator to device-level gathers
                      (bench.py: amr_allgather on a plan's device buffers)
      StoreTransport  the same operations through the store (CPU, tests)
    A transport is anything with those methods: tests/test_multi.py drives
    the packing below with a torch.distributed (gloo) one of its own.
  * ShardLayout: which streams a rank owns and the fixed-size wire format of
    the gather, including several global batches per launch (a strong-scaling
    shard too small to fill a GPU takes C consecutive batches' shards):
      payload [world][C * B_slot][cap] uint8   decoded bytes, zero padded
      lengths [world][C * B_slot]      int64   bytes per stream (-1 = padding)
  * demod_sharded / demodulate_sharded: the sharded form of the *_batch
    demodulators (decoder.decode_from_buffer_batch(..., transport=) uses it).

Reference: the reference is single-process (decoder.py:417-464 demodulates
one capture per call); this module is the batched, sharded form of that call
for BASELINE configs[3]/[4] (a global batch of 8192 over 8 GPUs).
"""
from __future__ import annotations

import os
import socket
import struct
import threading
import time

import numpy as np


# ---------------------------------------------------------------------------
# shard arithmetic and the wire format
def shard_range(n_streams: int, rank: int, world: int):
    """Contiguous, balanced [lo, hi) of the streams owned by `rank`."""
    base, extra = divmod(n_streams, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def max_local(n_streams: int, world: int) -> int:
    return -(-n_streams // world)


def pack(outs, max_streams: int, cap: int):
    """list[bytes] -> (payload [max_streams][cap] uint8, lengths [max_streams] int64)."""
    payload = np.zeros((max_streams, cap), np.uint8)
    lengths = np.full(max_streams, -1, np.int64)
    for i, o in enumerate(outs):
        if len(o) > cap:
            raise ValueError("decoded stream longer than the gather capacity")
        payload[i, :len(o)] = np.frombuffer(o, np.uint8)
        lengths[i] = len(o)
    return payload, lengths


def unpack(payload: np.ndarray, lengths: np.ndarray):
    """Inverse of pack over the gathered [world][max_local] layout, rank-major."""
    out = []
    for p, ln in zip(payload.reshape(-1, payload.shape[-1]), lengths.reshape(-1)):
        if ln >= 0:
            out.append(p[:ln].tobytes())
    return out


class ShardLayout:
    """The sharding of `steps` consecutive global batches of n_streams each
    over `world` ranks, all of a rank's shards in one launch.

    rank r owns streams shard_range(n_streams, r, world) of every step; its
    launch holds them step-major (steps * shard rows); its gather slot is
    steps * B_slot rows (B_slot = ceil(n_streams / world)), padded at the end."""

    def __init__(self, n_streams: int, world: int, steps: int = 1):
        self.n_streams, self.world, self.steps = int(n_streams), int(world), max(1, int(steps))
        self.b_slot = max_local(self.n_streams, self.world) if self.n_streams else 0
        self.rows = self.steps * self.b_slot

    def shard(self, rank: int):
        return shard_range(self.n_streams, rank, self.world)

    def shard_size(self, rank: int) -> int:
        lo, hi = self.shard(rank)
        return hi - lo

    def launch_rows(self, rank: int) -> int:
        return self.steps * self.shard_size(rank)

    def local_rows(self, x_steps, rank: int) -> np.ndarray:
        """The rank's launch input: its shard of every step's [n_streams, N] batch, step-major."""
        lo, hi = self.shard(rank)
        return np.concatenate([np.asarray(x)[lo:hi] for x in x_steps]) if x_steps else np.zeros((0, 0))

    def pack(self, outs, cap: int):
        """The rank's launch outputs (list[bytes], step-major) -> its gather slot."""
        return pack(outs, self.rows, cap)

    def unpack(self, payload: np.ndarray, lengths: np.ndarray):
        """Gathered [world][rows][cap] + [world][rows] -> list[bytes] of every step,
        step-major, each in global stream order (rank r's rows of step c are
        c * shard_size(r) .. (c+1) * shard_size(r) - 1 of slot r)."""
        payload = payload.reshape(self.world, self.rows, -1)
        lengths = lengths.reshape(self.world, self.rows)
        out = []
        for c in range(self.steps):
            for r in range(self.world):
                n = self.shard_size(r)
                for i in range(c * n, (c + 1) * n):
                    ln = int(lengths[r, i])
                    if ln < 0:
                        raise ValueError(f"gathered slot {r} row {i} is padding (no stream)")
                    out.append(payload[r, i, :ln].tobytes())
        return out


# ---------------------------------------------------------------------------
# bootstrap stores
class FileStore:
    """Key -> bytes in a directory shared by the ranks of one node.  set is an
    atomic rename; get polls until the key appears (or `timeout` s)."""

    def __init__(self, path: str, timeout: float = 300.0):
        self.path, self.timeout = path, timeout
        os.makedirs(path, exist_ok=True)

    def _file(self, key: str) -> str:
        return os.path.join(self.path, key.replace("/", "__"))

    def set(self, key: str, value: bytes):
        f = self._file(key)
        tmp = f"{f}.tmp{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(value)
        os.replace(tmp, f)

    def get(self, key: str) -> bytes:
        f = self._file(key)
        t0 = time.monotonic()
        delay = 20e-6
        while not os.path.exists(f):
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"FileStore: no key {key!r} in {self.path} after {self.timeout} s")
            time.sleep(delay)
            delay = min(2e-3, delay * 2)
        with open(f, "rb") as fh:
            return fh.read()

    def delete(self, key: str):
        try:
            os.remove(self._file(key))
        except FileNotFoundError:
            pass

    def close(self, owner: bool = False):
        if owner:
            import shutil
            shutil.rmtree(self.path, ignore_errors=True)


class _TcpServer(threading.Thread):
    def __init__(self, host: str, port: int):
        super().__init__(daemon=True)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self.data, self.cv, self.stop = {}, threading.Condition(), False

    def run(self):
        while not self.stop:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn):
        with conn:
            try:
                while True:
                    op, key, val = _recv_msg(conn)
                    if op == b"S":
                        with self.cv:
                            self.data[key] = val
                            self.cv.notify_all()
                        _send_msg(conn, b"K", key, b"")
                    elif op == b"G":
                        with self.cv:
                            self.cv.wait_for(lambda: key in self.data or self.stop)
                            v = self.data.get(key, b"")
                        _send_msg(conn, b"V", key, v)
                    elif op == b"D":
                        with self.cv:
                            self.data.pop(key, None)
                        _send_msg(conn, b"K", key, b"")
            except (ConnectionError, OSError):
                return

    def shutdown(self):
        self.stop = True
        with self.cv:
            self.cv.notify_all()
        try:
            self.sock.close()
        except OSError:
            pass


def _send_msg(conn, op: bytes, key: str | bytes, val: bytes):
    k = key.encode() if isinstance(key, str) else key
    conn.sendall(op + struct.pack("<IQ", len(k), len(val)) + k + val)


def _recv_exact(conn, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = conn.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("store connection closed")
        buf += chunk
    return bytes(buf)


def _recv_msg(conn):
    hdr = _recv_exact(conn, 13)
    op, (kl, vl) = hdr[:1], struct.unpack("<IQ", hdr[1:])
    key = _recv_exact(conn, kl).decode()
    return op, key, _recv_exact(conn, vl)


class TcpStore:
    """Key -> bytes held by rank 0 (`is_server`), served over TCP."""

    def __init__(self, host: str, port: int, is_server: bool, timeout: float = 300.0):
        self.server = _TcpServer(host, port) if is_server else None
        if self.server:
            self.server.start()
            port = self.server.port
        self.host, self.port = host, port
        t0 = time.monotonic()
        while True:
            try:
                self.conn = socket.create_connection((host, port), timeout=timeout)
                break
            except OSError:
                if time.monotonic() - t0 > timeout:
                    raise
                time.sleep(0.05)
        self.conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.lock = threading.Lock()

    def set(self, key: str, value: bytes):
        with self.lock:
            _send_msg(self.conn, b"S", key, bytes(value))
            _recv_msg(self.conn)

    def get(self, key: str) -> bytes:
        with self.lock:
            _send_msg(self.conn, b"G", key, b"")
            return _recv_msg(self.conn)[2]

    def delete(self, key: str):
        with self.lock:
            _send_msg(self.conn, b"D", key, b"")
            _recv_msg(self.conn)

    def close(self, owner: bool = False):
        try:
            self.conn.close()
        except OSError:
            pass
        if self.server and owner:
            self.server.shutdown()


def _parent_instance() -> str:
    """The parent process's pid and start time (/proc/<ppid>/stat field 22):
    the ranks of one torch.distributed.run launch, or of one multiprocessing
    pool, share it, and a later launch cannot -- even one whose agent got the
    same pid -- so a store left behind by a crashed run is never read again
    (ADVICE r3)."""
    ppid = os.getppid()
    try:
        with open(f"/proc/{ppid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return f"{ppid}_{fields[19]}"
    except (OSError, IndexError):
        return str(ppid)


def store_from_env(rank: int, world: int):
    """The bootstrap store: AMR_STORE=file:<dir> or tcp://<host>:<port> (rank 0
    serves), else a FileStore under the temp directory named after MASTER_PORT,
    the torchrun run id and the parent process instance (pid + start time)."""
    spec = os.environ.get("AMR_STORE", "")
    if spec.startswith("tcp://"):
        host, port = spec[6:].rsplit(":", 1)
        return TcpStore(host, int(port), is_server=rank == 0)
    if spec.startswith("file:"):
        return FileStore(spec[5:])
    import tempfile
    tag = (f"amr_store_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('TORCHELASTIC_RUN_ID', '')}_"
           f"{_parent_instance()}_{world}")
    return FileStore(os.path.join(tempfile.gettempdir(), tag))


def release_store(store, rank: int, world: int):
    """Every rank is done with the store: ranks > 0 say so and leave; rank 0
    waits for all of them, then removes it (nobody reads a key after saying
    done, so no rank can be left polling a deleted key)."""
    if rank == 0:
        for r in range(1, world):
            store.get(f"done/{r}")
    else:
        store.set(f"done/{rank}", b"")
    store.close(owner=rank == 0)


# ---------------------------------------------------------------------------
# transports
class StoreTransport:
    """all_gather / max / barrier through the bootstrap store (host bytes; CPU)."""

    def __init__(self, store, rank: int, world: int):
        self.store, self.rank, self.world = store, int(rank), int(world)
        self.seq = 0

    def _exchange(self, blob: bytes):
        tag = f"x{self.seq}"
        self.seq += 1
        self.store.set(f"{tag}/{self.rank}", blob)
        parts = [self.store.get(f"{tag}/{r}") for r in range(self.world)]
        # every rank has posted this exchange, so every rank is done reading
        # the previous one: this rank's key of it can go (a long-lived
        # transport keeps at most two exchanges in the store)
        if self.seq >= 2:
            self.store.delete(f"x{self.seq - 2}/{self.rank}")
        return parts

    def all_gather(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a)
        parts = self._exchange(a.tobytes())
        return np.stack([np.frombuffer(p, a.dtype).reshape(a.shape) for p in parts])

    def max(self, v: float) -> float:
        return float(self.all_gather(np.array([v], np.float64)).max())

    def barrier(self):
        self._exchange(b"")

    def close(self):
        release_store(self.store, self.rank, self.world)


class RcclTransport:
    """RCCL through libamr.so: the unique id from rank 0 via the store, one
    communicator per process on GPU `device`.  all_gather stages host arrays
    through the comm's device buffer (amr_comm_allgather_host); device-level
    gathers ordered against a plan's stream take `comm` directly
    (amr_allgather / amr_fsk_allgather)."""

    def __init__(self, store, rank: int, world: int, device: int):
        import ctypes
        import _amr
        self.rank, self.world, self.device = int(rank), int(world), int(device)
        self._amr, self._ct = _amr, ctypes
        L = _amr.lib()
        _amr.check(L.amr_set_device(self.device))
        uid = (ctypes.c_uint8 * 128)()
        if self.rank == 0:
            _amr.check(L.amr_comm_unique_id(uid))
            store.set("rccl_uid", bytes(uid))
        else:
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(store.get("rccl_uid"))
        self.comm = ctypes.c_void_p()
        _amr.check(L.amr_comm_create(ctypes.byref(self.comm), uid, self.world, self.rank, self.device))
        self.store = store
        self.barrier()                         # every rank holds the id: the store may go

    def all_gather(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a)
        out = np.empty((self.world,) + a.shape, a.dtype)
        if a.nbytes:
            self._amr.check(self._amr.lib().amr_comm_allgather_host(self.comm, self._amr.ptr(a), self._amr.ptr(out),
                                                                    a.nbytes))
        return out

    def max(self, v: float) -> float:
        a = np.array([v], np.float64)
        self._amr.check(self._amr.lib().amr_comm_allreduce_max(self.comm, self._amr.ptr(a), 1))
        return float(a[0])

    def barrier(self):
        self.max(0.0)

    def close(self):
        if self.comm:
            self.barrier()
            self._amr.lib().amr_comm_destroy(self.comm)
            self.comm = None
            release_store(self.store, self.rank, self.world)


def transport_from_env(device=None, kind: str = "rccl"):
    """RANK / WORLD_SIZE / LOCAL_RANK from the launcher's environment -> a transport."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
    store = store_from_env(rank, world)
    if kind == "rccl":
        return RcclTransport(store, rank, world, dev)
    return StoreTransport(store, rank, world)


# ---------------------------------------------------------------------------
# the sharded demodulation
def gather_outputs(outs, layout: ShardLayout, cap: int, transport):
    """This rank's launch outputs -> every step's outputs of the whole
    global batch (list[bytes], step-major), on every rank."""
    payload, lengths = layout.pack(outs, cap)
    gp = transport.all_gather(payload)
    gl = transport.all_gather(lengths)
    return layout.unpack(gp, gl)


def demod_sharded(x, demod_batch, transport, cap: int | None = None, steps=None):
    """Demodulate this rank's shard of x with demod_batch and gather the result.

    x          : [B, N] the global batch (rows outside the rank's shard are not
                 read), or a list of `steps` such batches demodulated as one
                 launch per rank (ShardLayout with steps > 1)
    demod_batch: callable([b, N]) -> list[bytes]  (modem.qpsk_demodulate_batch etc.)
    transport  : RcclTransport / StoreTransport / any object with rank, world, all_gather
    cap        : gather capacity per stream (default: the longest local output, agreed by max)
    Returns the decoded bytes of every stream (every step), in global order, on every rank."""
    xs = list(x) if steps is not None or isinstance(x, (list, tuple)) else [x]
    n = np.asarray(xs[0]).shape[0] if xs else 0
    layout = ShardLayout(n, transport.world, len(xs))
    local = layout.local_rows(xs, transport.rank)
    err = None
    try:
        outs = demod_batch(local) if len(local) else []
    except Exception as e:                     # reported on every rank below
        outs, err = [], e
    # one small collective carries whether any rank failed and the longest
    # local output (the gather's capacity): a rank whose demodulation raised
    # still joins it, so no rank is left waiting in the gather for it
    st = transport.all_gather(np.array([err is not None, max((len(o) for o in outs), default=0)], np.int64))
    failed = [int(r) for r in np.flatnonzero(st[:, 0])]
    if failed:
        if err is not None:
            raise err
        raise RuntimeError(f"demodulation failed on rank(s) {failed}")
    if cap is None:
        cap = int(st[:, 1].max())
    return gather_outputs(outs, layout, max(1, cap), transport)


def demodulate_sharded(kind: str, x: np.ndarray, baud, transport, **kw):
    """modem.{qpsk,bpsk,fsk}_demodulate_batch over the ranks: each rank
    demodulates its shard of the global [B, N] batch on its GPU, the decoded
    bytes are all-gathered; every rank returns the global list[bytes]."""
    import modem
    fn = {"qpsk": modem.qpsk_demodulate_batch, "bpsk": modem.bpsk_demodulate_batch,
          "fsk": modem.fsk_demodulate_batch}[kind]
    return demod_sharded(np.asarray(x), lambda xs: fn(xs, baud=baud, **kw), transport)


def digests(rows: np.ndarray, lens: np.ndarray, sync: np.ndarray = None) -> np.ndarray:
    """Per-stream 8-byte digest of decoded bytes + length (+ the sync index,
    SURVEY §8(e)'s third gathered array, when given) -- the gather check, [n] int64."""
    import hashlib
    return np.array([int.from_bytes(hashlib.blake2b(rows[i, :max(0, int(lens[i]))].tobytes()
                                                    + int(lens[i]).to_bytes(8, "little", signed=True)
                                                    + (b"" if sync is None else
                                                       int(sync[i]).to_bytes(8, "little", signed=True)),
                                                    digest_size=8).digest(), "little", signed=True)
                     for i in range(rows.shape[0])], np.int64)


def gather_check(gathered_payload: np.ndarray, gathered_lengths: np.ndarray, own_payload: np.ndarray,
                 own_lengths: np.ndarray, layout: ShardLayout, transport, gathered_sync: np.ndarray = None,
                 own_sync: np.ndarray = None) -> list:
    """Rank r's slice of the gathered buffer must equal rank r's own launch
    output, stream for stream (its real rows; the slot padding is not
    compared): bytes, lengths and, when given, sync indices.  Every rank
    checks every slice against digests all-gathered from the ranks
    themselves; returns the sorted ranks whose slices differ (as seen by any
    rank)."""
    n_own = layout.launch_rows(transport.rank)
    mine = np.zeros(layout.rows, np.int64)
    mine[:n_own] = digests(own_payload[:n_own], own_lengths[:n_own], None if own_sync is None else own_sync[:n_own])
    own_all = transport.all_gather(mine)
    bad = np.zeros(transport.world, np.float64)
    for r in range(transport.world):
        n = layout.launch_rows(r)
        got = digests(gathered_payload[r][:n], gathered_lengths[r][:n],
                      None if gathered_sync is None else gathered_sync[r][:n])
        bad[r] = float(not np.array_equal(got, own_all[r][:n]))
    flags = transport.all_gather(bad)
    return sorted(int(r) for r in np.flatnonzero(flags.max(axis=0) > 0))
