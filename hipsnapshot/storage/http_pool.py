"""Blocking keep-alive HTTP/1.1 client for bulk object-store transfers.

The S3 plugin's payload path (reference: aiobotocore ``put_object`` /
ranged ``get_object``, `/root/reference/torchsnapshot/storage_plugins/s3.py:39-66`)
moves checkpoint blobs of 64 MiB-512 MiB.  Through aiohttp every GET body is
first assembled in a ``bytes`` object (``await resp.read()``) and copied
again into its destination, and every byte passes the one event-loop
thread.  Here each transfer runs on a worker thread over a blocking socket:

* request bodies go out with ``sendall(memoryview)`` straight from the staged
  (pinned) buffer -- no ``tobytes()``;
* response bodies land with ``recv_into`` directly in the caller's destination
  slice (pinned read buffer of the consumer) -- the kernel copy is the only
  copy;
* the socket syscalls release the GIL, so ``max_conns`` parts move in
  parallel on as many cores.

TLS (``https://``) wraps the same sockets with ``ssl``.  Only what S3 needs
is implemented: Content-Length and chunked responses, keep-alive reuse.
"""

from __future__ import annotations

import queue
import socket
import ssl
from typing import Dict, Optional, Tuple, Union

Body = Union[bytes, bytearray, memoryview, None]


class HTTPError(OSError):
    pass


class _Conn:
    __slots__ = ("sock", "buf")

    def __init__(self, sock: socket.socket) -> None:
        self.sock = sock
        self.buf = bytearray()  # bytes received past the last response

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class HTTPPool:
    def __init__(self, scheme: str, host: str, port: Optional[int] = None,
                 max_conns: int = 16, timeout: float = 300.0) -> None:
        self.scheme = scheme
        self.host = host
        self.port = port or (443 if scheme == "https" else 80)
        default = 443 if scheme == "https" else 80
        self.host_header = host if self.port == default else f"{host}:{self.port}"
        self.timeout = timeout
        self._idle: "queue.LifoQueue[_Conn]" = queue.LifoQueue()
        self._ssl = ssl.create_default_context() if scheme == "https" else None
        self.max_conns = max_conns

    # -- connections --------------------------------------------------------------

    def _connect(self) -> _Conn:
        sock = socket.create_connection((self.host, self.port), timeout=self.timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        for opt in (socket.SO_SNDBUF, socket.SO_RCVBUF):
            try:
                sock.setsockopt(socket.SOL_SOCKET, opt, 8 << 20)
            except OSError:
                pass
        if self._ssl is not None:
            sock = self._ssl.wrap_socket(sock, server_hostname=self.host)
        return _Conn(sock)

    def _acquire(self) -> Tuple[_Conn, bool]:
        try:
            return self._idle.get_nowait(), True
        except queue.Empty:
            return self._connect(), False

    def close(self) -> None:
        while True:
            try:
                self._idle.get_nowait().close()
            except queue.Empty:
                return

    # -- one request ----------------------------------------------------------------

    def request(self, method: str, target: str, headers: Dict[str, str], body: Body = None,
                dest: Optional[memoryview] = None) -> Tuple[int, Dict[str, str], bytes, int]:
        """Send one request; returns (status, lower-cased headers, body bytes,
        bytes written into ``dest``).  A 2xx body whose length fits ``dest``
        is received straight into it (then the returned body is empty).

        A reused keep-alive connection that the server closed meanwhile is
        retried once on a fresh one (the request was not processed)."""
        for _ in (0, 1):
            conn, reused = self._acquire()
            try:
                out = self._exchange(conn, method, target, headers, body, dest)
            except (ConnectionError, ssl.SSLError) as e:
                conn.close()
                if not reused or getattr(e, "_hs_response_started", False):
                    raise
                continue  # a stale keep-alive connection: once more on a new one
            except BaseException:
                conn.close()
                raise
            status, hdrs, data, n, keep = out
            if keep:
                self._idle.put(conn)
            else:
                conn.close()
            return status, hdrs, data, n
        raise HTTPError("unreachable")  # pragma: no cover

    def _exchange(self, conn: _Conn, method: str, target: str, headers: Dict[str, str],
                  body: Body, dest: Optional[memoryview]):
        mv = memoryview(body).cast("B") if body is not None else None
        lines = [f"{method} {target} HTTP/1.1", f"Host: {self.host_header}"]
        have_len = False
        for k, v in headers.items():
            if k.lower() == "host":
                continue
            have_len |= k.lower() == "content-length"
            lines.append(f"{k}: {v}")
        if not have_len and (mv is not None or method in ("PUT", "POST")):
            lines.append(f"Content-Length: {mv.nbytes if mv is not None else 0}")
        head = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
        sock = conn.sock
        if mv is not None and mv.nbytes <= 64 << 10:
            sock.sendall(head + mv.tobytes())
        else:
            sock.sendall(head)
            if mv is not None:
                sock.sendall(mv)
        try:
            return self._read_response(conn, method, dest)
        except ConnectionError as e:
            e._hs_response_started = bool(conn.buf)  # type: ignore[attr-defined]
            raise

    def _fill(self, conn: _Conn, need: int) -> None:
        while len(conn.buf) < need:
            chunk = conn.sock.recv(max(65536, need - len(conn.buf)))
            if not chunk:
                raise ConnectionResetError("connection closed by the server")
            conn.buf += chunk

    def _read_line(self, conn: _Conn) -> bytes:
        while True:
            i = conn.buf.find(b"\r\n")
            if i >= 0:
                line = bytes(conn.buf[:i])
                del conn.buf[: i + 2]
                return line
            chunk = conn.sock.recv(65536)
            if not chunk:
                raise ConnectionResetError("connection closed by the server")
            conn.buf += chunk

    def _read_response(self, conn: _Conn, method: str, dest: Optional[memoryview]):
        status_line = self._read_line(conn)
        parts = status_line.split(b" ", 2)
        if len(parts) < 2 or not parts[0].startswith(b"HTTP/"):
            raise HTTPError(f"bad status line {status_line[:80]!r}")
        status = int(parts[1])
        hdrs: Dict[str, str] = {}
        while True:
            line = self._read_line(conn)
            if not line:
                break
            k, _, v = line.decode("latin-1").partition(":")
            hdrs[k.strip().lower()] = v.strip()
        keep = hdrs.get("connection", "").lower() != "close"
        if method == "HEAD" or status in (204, 304) or 100 <= status < 200:
            return status, hdrs, b"", 0, keep
        if hdrs.get("transfer-encoding", "").lower() == "chunked":
            data = bytearray()
            while True:
                size = int(self._read_line(conn).split(b";")[0], 16)
                if size == 0:
                    while self._read_line(conn):
                        pass
                    break
                self._fill(conn, size + 2)
                data += conn.buf[:size]
                del conn.buf[: size + 2]
            if dest is not None and 200 <= status < 300 and len(data) <= dest.nbytes:
                dest[: len(data)] = data
                return status, hdrs, b"", len(data), keep
            return status, hdrs, bytes(data), 0, keep
        if "content-length" not in hdrs:
            # body until close
            data = bytearray(conn.buf)
            conn.buf.clear()
            while True:
                chunk = conn.sock.recv(1 << 20)
                if not chunk:
                    break
                data += chunk
            return status, hdrs, bytes(data), 0, False
        n = int(hdrs["content-length"])
        if dest is not None and 200 <= status < 300 and n <= dest.nbytes:
            got = min(len(conn.buf), n)
            if got:
                dest[:got] = conn.buf[:got]
                del conn.buf[:got]
            view = dest[got:n]  # the rest of the body, straight from the socket
            # plain TCP: one blocking syscall for the whole rest (GIL released
            # once, not per 64 KiB segment); TLS sockets take no flags
            flags = 0 if self._ssl is not None else socket.MSG_WAITALL
            while got < n:
                r = conn.sock.recv_into(view, n - got, flags)
                if r == 0:
                    raise ConnectionResetError("connection closed mid-body")
                view = view[r:]
                got += r
            return status, hdrs, b"", n, keep
        self._fill(conn, n)
        data = bytes(conn.buf[:n])
        del conn.buf[:n]
        return status, hdrs, data, 0, keep
