"""TCP compatibility transport: the reference's wire protocol, for cross-host or
plumbing use (NOT the MI355X hot path -- that is the RCCL all-reduce).

Framing (client1.py:246-273, server.py:29-55), kept byte-compatible:
  sender   : b"<decimal size>\\n" + payload in 1 MiB sendall() chunks
             [server side: shutdown(SHUT_WR)]
  receiver : header read byte-by-byte to b"\\n"; recv(min(4 MiB, remaining)) into a
             preallocated buffer (the reference's ``data += packet`` is quadratic);
             then sends b"RECEIVED"
  sender   : recv(1024) == b"RECEIVED" -> success
Ports: uploads to 12345, downloads from 12346 (server.py:11-12).

Deliberate differences:
  * payload codec: gzip(torch.save(state_dict)) decoded with
    ``torch.load(weights_only=True)`` -- never unpickle bytes from a socket
    (the reference sends gzip(pickle.dumps(state_dict)) and decodes it with
    pickle.loads, client1.py:228-243).  ONLY THE FRAMING is compatible: this
    server cannot decode a reference client's payload and a reference server
    cannot decode ours.  gzip level defaults to 1, not 9 (the level-9 compress is
    11 s of the reference's ~20 s round);
  * download requests start with b"GET\\n" so a readiness probe (the reference's
    wait_for_server) is never mistaken for a client (the WinError 10053 bug,
    SURVEY 5.3); ``strict_compat=True`` only drops that handshake (the
    reference's download framing), it does not change the payload codec;
  * a failed or timed-out accept counts against the server's error budget and
    the round carries on with the clients that did connect (the reference's
    upload accept raises uncaught after 300 s, server.py:119,126);
  * server-side client ids follow the order uploads complete, and are logged.
"""
from __future__ import annotations

import gzip
import io
import socket
import threading
import time
from typing import Callable, Dict, List, Optional

import torch

CHUNK = 1024 * 1024
RECV_CHUNK = 4 * 1024 * 1024
ACK = b"RECEIVED"
HELLO = b"GET\n"
PORT_RECEIVE = 12345
PORT_SEND = 12346
TIMEOUT = 300.0
NUM_CLIENTS = 2


# ------------------------------------------------------------------ codec
def encode_state(state: Dict[str, torch.Tensor], level: int = 1) -> bytes:
    buf = io.BytesIO()
    torch.save({k: v.detach().cpu() for k, v in state.items()}, buf)
    return gzip.compress(buf.getvalue(), compresslevel=level)


def decode_state(data: bytes) -> Dict[str, torch.Tensor]:
    return torch.load(io.BytesIO(gzip.decompress(data)), map_location="cpu", weights_only=True)


# ------------------------------------------------------------------ framing
def send_chunked_data(sock: socket.socket, data: bytes, chunk_size: int = CHUNK, shutdown: bool = False) -> bool:
    sock.sendall(f"{len(data)}\n".encode())
    mv = memoryview(data)
    for i in range(0, len(data), chunk_size):
        sock.sendall(mv[i:i + chunk_size])
    if shutdown:
        sock.shutdown(socket.SHUT_WR)
    ack = sock.recv(1024)
    return ack == ACK


def _read_header(sock: socket.socket) -> int:
    hdr = bytearray()
    while True:
        b = sock.recv(1)
        if not b:
            raise ConnectionError("peer closed before header")
        if b == b"\n":
            return int(hdr.decode())
        hdr += b


def receive_chunked_data(sock: socket.socket) -> bytes:
    total = _read_header(sock)
    buf = bytearray(total)
    view = memoryview(buf)
    got = 0
    while got < total:
        n = sock.recv_into(view[got:], min(RECV_CHUNK, total - got))
        if n == 0:
            break
        got += n
    sock.sendall(ACK)
    if got != total:
        raise ConnectionError(f"short payload: {got}/{total} bytes")
    return bytes(buf)


# ------------------------------------------------------------------ client side
def wait_for_server(host: str, port: int, timeout: float = TIMEOUT, interval: float = 1.0) -> bool:
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            with socket.create_connection((host, port), timeout=3):
                return True
        except OSError:
            time.sleep(interval)
    return False


def send_model(state: Dict[str, torch.Tensor], host: str = "localhost", port: int = PORT_RECEIVE,
               level: int = 1, timeout: float = TIMEOUT, log=None) -> bool:
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.settimeout(timeout)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 * 1024 * 1024)
            s.connect((host, port))
            payload = encode_state(state, level)
            ok = send_chunked_data(s, payload)
            if log:
                log.phase(f"sent {len(payload) / 1e6:.1f} MB model (ack={'ok' if ok else 'bad'})")
            return ok
    except OSError as e:
        if log:
            log.phase(f"[ERROR] send failed: {e}")
        return False


def receive_aggregated_model(host: str = "localhost", port: int = PORT_SEND, max_retries: int = 5,
                             timeout: float = TIMEOUT, strict_compat: bool = False, log=None):
    for attempt in range(max_retries):
        if not wait_for_server(host, port, timeout):
            continue
        try:
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                s.settimeout(timeout)
                s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 * 1024 * 1024)
                s.connect((host, port))
                if not strict_compat:
                    s.sendall(HELLO)
                data = receive_chunked_data(s)
                return decode_state(data)
        except (OSError, ConnectionError) as e:
            if log:
                log.phase(f"[ERROR] receive attempt {attempt + 1} failed: {e}")
    return None


# ------------------------------------------------------------------ server side
class FedAvgServer:
    """server.py equivalent: gather N uploads, FedAvg, broadcast the mean back."""

    def __init__(self, num_clients: int = NUM_CLIENTS, host: str = "localhost", port_receive: int = PORT_RECEIVE,
                 port_send: int = PORT_SEND, timeout: float = TIMEOUT, strict_compat: bool = False,
                 aggregate: Optional[Callable] = None, save_path: Optional[str] = None, log=None, level: int = 1):
        from .fedavg import aggregate_state_dicts
        self.n, self.host = num_clients, host
        self.port_receive, self.port_send = port_receive, port_send
        self.timeout, self.strict = timeout, strict_compat
        self.aggregate = aggregate or (lambda states: aggregate_state_dicts(states, num_clients=num_clients))
        self.save_path, self.log, self.level = save_path, log, level
        self.received: List[Dict[str, torch.Tensor]] = []
        self.lock = threading.Lock()
        self.ready = threading.Event()

    def _handle(self, conn: socket.socket, addr, cid: int):
        try:
            conn.settimeout(self.timeout)
            state = decode_state(receive_chunked_data(conn))
            with self.lock:
                self.received.append(state)
            if self.log:
                self.log.phase(f"[RECV] model from client {cid} {addr}")
        except Exception as e:  # pragma: no cover - network errors
            if self.log:
                self.log.phase(f"[ERROR] client {cid} {addr}: {e}")
        finally:
            conn.close()

    def gather(self, max_errors: int = 5):
        """Accept up to N uploads; an accept that times out or fails counts against
        ``max_errors`` (the reference's retry budget, server.py:92-112) instead of aborting the
        round, so the clients that did connect are still aggregated / answered."""
        errors = 0
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as srv:
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((self.host, self.port_receive))
            srv.listen(self.n)
            srv.settimeout(self.timeout)
            self.ready.set()
            threads = []
            while len(threads) < self.n and errors < max_errors:
                try:
                    conn, addr = srv.accept()
                except OSError as e:  # socket.timeout is an OSError
                    errors += 1
                    if self.log:
                        self.log.phase(f"[ERROR] accept failed ({errors}/{max_errors}): {e}")
                    continue
                t = threading.Thread(target=self._handle, args=(conn, addr, len(threads)))
                t.start()
                threads.append(t)
            for t in threads:
                t.join()
        if self.log and len(threads) < self.n:
            self.log.phase(f"[ERROR] gave up after {errors} accept errors: {len(threads)}/{self.n} clients connected")
        return self.received

    def broadcast(self, state: Dict[str, torch.Tensor], max_errors: int = 5) -> int:
        payload = encode_state(state, self.level)
        served, errors = 0, 0
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as srv:
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((self.host, self.port_send))
            srv.listen(self.n)
            srv.settimeout(self.timeout)
            while served < self.n and errors < max_errors:
                try:
                    conn, addr = srv.accept()
                except OSError as e:
                    errors += 1
                    if self.log:
                        self.log.phase(f"[ERROR] accept failed ({errors}/{max_errors}): {e}")
                    continue
                try:
                    conn.settimeout(self.timeout)
                    if not self.strict:
                        req = conn.recv(len(HELLO))
                        if req != HELLO:  # readiness probe: not a client
                            conn.close()
                            continue
                    if send_chunked_data(conn, payload, shutdown=True):
                        served += 1
                        if self.log:
                            self.log.phase(f"[SEND] aggregated model to {addr}")
                    else:
                        errors += 1
                except OSError as e:
                    errors += 1
                    if self.log:
                        self.log.phase(f"[ERROR] send to {addr}: {e}")
                finally:
                    conn.close()
        if self.log and served < self.n:
            self.log.phase(f"[ERROR] served {served}/{self.n} clients before giving up ({errors} errors)")
        return served

    def run_round(self):
        states = self.gather()
        agg = self.aggregate(states)
        if agg is None:
            if self.log:
                self.log.phase(f"[ERROR] expected {self.n} models, got {len(states)}")
            return None
        if self.save_path:
            torch.save(agg, self.save_path)
        self.broadcast(agg)
        return agg
