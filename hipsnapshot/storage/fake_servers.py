"""Fake S3 and GCS servers for tests and benchmarks.

There is no network on the build or GPU boxes, so the S3/GCS plugins are
exercised end to end against these: the fake S3 server VERIFIES every SigV4
signature (recomputed from the raw request with the shared secret) and
implements PUT/GET(Range)/HEAD/DELETE, multipart uploads and ListObjectsV2
on a threaded HTTP/1.1 server that can also run as its own process
(``FakeS3Process``); the
fake GCS server implements media + resumable uploads (308 / Range protocol),
ranged ``alt=media`` downloads and DELETE.  Both support fault injection
(``fail_next(n, status)``) to test the retry paths.
"""

from __future__ import annotations

import asyncio
import datetime as _dt
import random
import re
import threading
import uuid
from typing import Dict, Optional

from aiohttp import web

from .s3 import sigv4_headers


class _ServerThread:
    def __init__(self) -> None:
        self.loop = asyncio.new_event_loop()
        self.port: Optional[int] = None
        self._runner = None
        self._thread = threading.Thread(target=self.loop.run_forever, daemon=True)
        self.fail_queue: list = []
        self.requests = 0
        self.fail_rate = 0.0
        self.injected = 0  # requests failed by fail_randomly
        self._fail_rng = random.Random(0)

    def fail_next(self, n: int = 1, status: int = 503) -> None:
        self.fail_queue.extend([status] * n)

    def fail_randomly(self, rate: float, seed: int = 0) -> None:
        """Fail each later request with probability ``rate`` (a transient
        408 / 429 / 500 / 503, seeded): a flaky service for retry tests."""
        self.fail_rate, self._fail_rng = float(rate), random.Random(seed)

    def _maybe_fail(self) -> Optional[web.Response]:
        self.requests += 1
        if self.fail_queue:
            return web.Response(status=self.fail_queue.pop(0), text="injected")
        if self.fail_rate and self._fail_rng.random() < self.fail_rate:
            self.injected += 1
            return web.Response(status=self._fail_rng.choice((408, 429, 500, 503)),
                                text="injected")
        return None

    def start(self, app: web.Application) -> "_ServerThread":
        self._thread.start()

        async def _up():
            self._runner = web.AppRunner(app, access_log=None)
            await self._runner.setup()
            site = web.TCPSite(self._runner, "127.0.0.1", 0)
            await site.start()
            return site._server.sockets[0].getsockname()[1]

        self.port = asyncio.run_coroutine_threadsafe(_up(), self.loop).result(30)
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def stop(self) -> None:
        async def _down():
            await self._runner.cleanup()

        asyncio.run_coroutine_threadsafe(_down(), self.loop).result(30)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._thread.join(10)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class _S3Object:
    """An object as the list of its uploaded bodies (a multipart object is
    never re-joined): ranged GETs send slices of the parts."""

    __slots__ = ("parts", "size")

    def __init__(self, parts) -> None:
        self.parts = list(parts)
        self.size = sum(len(p) for p in self.parts)

    def __eq__(self, other) -> bool:  # tests compare with bytes
        return bytes(self) == bytes(other)

    def __bytes__(self) -> bytes:
        return b"".join(bytes(p) for p in self.parts)

    def slices(self, lo: int, hi: int):
        pos = 0
        for p in self.parts:
            a, b = max(lo, pos), min(hi, pos + len(p))
            if b > a:
                yield memoryview(p)[a - pos: b - pos]
            pos += len(p)


class FakeS3Server:
    """S3 subset over a THREADED HTTP/1.1 server (one thread per keep-alive
    connection; bodies are received with ``readinto`` into one bytearray and
    sent from memoryview slices, so the server moves GB/s and the client is
    what gets measured).  Verifies every SigV4 signature.  Runs in-process
    (tests: ``objects`` / ``fail_next`` are visible) or in its own process
    (``FakeS3Process``, benchmarks: the snapshot process's GIL is not
    shared with the server)."""

    def __init__(self, access_key: str = "AKIDFAKE", secret: str = "fake-secret",
                 region: str = "us-east-1", port: int = 0) -> None:
        import http.server

        self.access_key, self.secret, self.region = access_key, secret, region
        self.objects: Dict[str, _S3Object] = {}
        self.uploads: Dict[str, Dict[int, bytearray]] = {}
        self.fail_queue: list = []
        self.requests = 0
        self.fail_rate = 0.0
        self.injected = 0  # requests failed by fail_randomly
        self._fail_rng = random.Random(0)
        self._lock = threading.Lock()
        server = self

        class Handler(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # quiet
                pass

            def setup(self):
                super().setup()
                import socket as _socket

                # the header write and the body write must not wait on the
                # client's delayed ACK (Nagle)
                self.connection.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
                for opt in (_socket.SO_SNDBUF, _socket.SO_RCVBUF):
                    try:
                        self.connection.setsockopt(_socket.SOL_SOCKET, opt, 8 << 20)
                    except OSError:
                        pass

            rbufsize = 0  # raw socket reads: no request body left in a Python buffer

            def _body(self):
                import numpy as _np
                import socket as _socket

                n = int(self.headers.get("Content-Length") or 0)
                buf = _np.empty(n, dtype=_np.uint8)  # no zero-fill pass
                view, got = memoryview(buf), 0
                while got < n:
                    # one blocking syscall for the whole body (GIL released):
                    # per-64 KiB recv calls convoyed the server's threads on
                    # the GIL at ~1 GB/s
                    r = self.connection.recv_into(view[got:], n - got, _socket.MSG_WAITALL)
                    if not r:
                        raise ConnectionResetError("client closed mid-body")
                    got += r
                return memoryview(buf)

            def _send(self, status: int, body=b"", headers=None) -> None:
                self.send_response(status)
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                if not any(k.lower() == "content-length" for k in (headers or {})):
                    self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                if body and self.command != "HEAD":
                    self.wfile.write(body)

            def _handle(self) -> None:
                body = self._body()
                resp = server._dispatch(self, body)
                if resp is not None:
                    self._send(*resp)

            do_GET = do_PUT = do_POST = do_DELETE = do_HEAD = _handle

        class Server(http.server.ThreadingHTTPServer):
            daemon_threads = True
            request_queue_size = 256

        self._httpd = Server(("127.0.0.1", port), Handler)
        self.port = self._httpd.server_address[1]
        self._thread = threading.Thread(target=self._httpd.serve_forever, daemon=True,
                                        kwargs={"poll_interval": 0.1})
        self._thread.start()

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def fail_next(self, n: int = 1, status: int = 503) -> None:
        self.fail_queue.extend([status] * n)

    def fail_randomly(self, rate: float, seed: int = 0) -> None:
        """Fail each later request with probability ``rate`` (a transient
        429 / 500 / 503, seeded): a flaky service for retry tests."""
        with self._lock:
            self.fail_rate, self._fail_rng = float(rate), random.Random(seed)

    def stop(self) -> None:
        self._httpd.shutdown()
        self._httpd.server_close()
        self._thread.join(10)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()

    # -- request handling ---------------------------------------------------------

    def _verify(self, h, path: str, query: Dict[str, str], body) -> Optional[tuple]:
        import hashlib

        auth = h.headers.get("Authorization", "")
        m = re.match(r"AWS4-HMAC-SHA256 Credential=([^/]+)/(\d{8})/([^/]+)/s3/aws4_request, "
                     r"SignedHeaders=([^,]+), Signature=([0-9a-f]{64})$", auth)
        if not m or m.group(1) != self.access_key:
            return 403, f"bad auth header {auth!r}".encode()
        signed = m.group(4).split(";")
        hdrs = {k: h.headers.get(k, "") for k in signed
                if k not in ("host", "x-amz-date", "x-amz-content-sha256")}
        now = _dt.datetime.strptime(h.headers["x-amz-date"], "%Y%m%dT%H%M%SZ").replace(
            tzinfo=_dt.timezone.utc)
        expect = sigv4_headers(h.command, h.headers["Host"], path, query, hdrs,
                               h.headers["x-amz-content-sha256"], self.access_key, self.secret,
                               m.group(3), now=now,
                               session_token=h.headers.get("x-amz-security-token"))
        if expect["Authorization"] != auth:
            return 403, b"SignatureDoesNotMatch"
        ph = h.headers["x-amz-content-sha256"]
        if ph != "UNSIGNED-PAYLOAD" and hashlib.sha256(body).hexdigest() != ph:
            return 400, b"XAmzContentSHA256Mismatch"
        return None

    def _dispatch(self, h, body: bytearray):
        from urllib.parse import parse_qsl, unquote, urlsplit

        u = urlsplit(h.path)
        path = unquote(u.path)
        q = dict(parse_qsl(u.query, keep_blank_values=True))
        with self._lock:
            self.requests += 1
            fail = self.fail_queue.pop(0) if self.fail_queue else None
            if fail is None and self.fail_rate and self._fail_rng.random() < self.fail_rate:
                fail = self._fail_rng.choice((429, 500, 503))
                self.injected += 1
        if fail is not None:
            return fail, b"injected"
        bad = self._verify(h, path, q, body)
        if bad is not None:
            return bad
        bucket, _, obj = path.lstrip("/").partition("/")
        m = h.command
        if not obj:  # bucket-level: ListObjectsV2
            if m == "GET" and q.get("list-type") == "2":
                prefix = q.get("prefix", "")
                with self._lock:
                    keys = sorted(k.split("/", 1)[1] for k in self.objects
                                  if k.startswith(f"{bucket}/{prefix}"))
                xml = "<ListBucketResult>" + "".join(f"<Contents><Key>{k}</Key></Contents>"
                                                     for k in keys) + "</ListBucketResult>"
                return 200, xml.encode(), {"Content-Type": "application/xml"}
            return 400, b""
        key = f"{bucket}/{obj}"
        if m == "POST" and "uploads" in q:
            uid = uuid.uuid4().hex
            with self._lock:
                self.uploads[uid] = {}
            return 200, (f"<InitiateMultipartUploadResult><UploadId>{uid}</UploadId>"
                         "</InitiateMultipartUploadResult>").encode()
        if m == "PUT" and "uploadId" in q:
            with self._lock:
                self.uploads[q["uploadId"]][int(q["partNumber"])] = body
            return 200, b"", {"ETag": f'"{q["partNumber"]}-{len(body)}"'}
        if m == "POST" and "uploadId" in q:
            nums = [int(n) for n in re.findall(r"<PartNumber>(\d+)</PartNumber>",
                                               bytes(body).decode())]
            with self._lock:
                parts = self.uploads.pop(q["uploadId"])
                self.objects[key] = _S3Object(parts[n] for n in nums)
            return 200, b"<CompleteMultipartUploadResult/>"
        if m == "DELETE" and "uploadId" in q:
            with self._lock:
                self.uploads.pop(q["uploadId"], None)
            return 204, b""
        if m == "PUT":
            with self._lock:
                self.objects[key] = _S3Object([body])
            return 200, b"", {"ETag": '"x"'}
        if m in ("GET", "HEAD"):
            with self._lock:
                o = self.objects.get(key)
            if o is None:
                return 404, b"NoSuchKey"
            if m == "HEAD":
                return 200, b"", {"Content-Length": str(o.size)}
            rng = h.headers.get("Range")
            lo, hi, status = 0, o.size, 200
            if rng:
                a, b = rng.split("=", 1)[1].split("-")
                lo, hi, status = int(a), min(int(b) + 1, o.size), 206
            h.send_response(status)
            h.send_header("Content-Length", str(max(hi - lo, 0)))
            if status == 206:
                h.send_header("Content-Range", f"bytes {lo}-{hi - 1}/{o.size}")
            h.end_headers()
            for sl in o.slices(lo, hi):
                h.wfile.write(sl)
            return None
        if m == "DELETE":
            with self._lock:
                self.objects.pop(key, None)
            return 204, b""
        return 405, b""


class FakeS3Process:
    """``FakeS3Server`` in its own process (``python -m
    hipsnapshot.storage.fake_servers s3``): benchmarks measure the client
    without sharing its GIL with the server.  ``stop()`` ends exactly the
    process this object started."""

    def __init__(self, access_key: str = "AKIDFAKE", secret: str = "fake-secret") -> None:
        import subprocess
        import sys

        self.proc = subprocess.Popen(
            [sys.executable, "-m", "hipsnapshot.storage.fake_servers", "s3", access_key, secret],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE)
        line = self.proc.stdout.readline().decode().split()
        if len(line) != 2 or line[0] != "PORT":
            self.proc.kill()
            raise RuntimeError(f"fake S3 process did not start: {line}")
        self.port = int(line[1])

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def stop(self) -> None:
        if self.proc.poll() is None:
            self.proc.stdin.close()  # the server exits when its stdin closes
            try:
                self.proc.wait(30)
            except Exception:  # noqa: BLE001
                self.proc.kill()
                self.proc.wait()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class FakeGCSServer(_ServerThread):
    def __init__(self, token: Optional[str] = "fake-token") -> None:
        super().__init__()
        self.token = token
        self.objects: Dict[str, bytes] = {}
        self.sessions: Dict[str, dict] = {}
        app = web.Application(client_max_size=1 << 40)
        app.router.add_post("/upload/storage/v1/b/{bucket}/o", self._upload)
        app.router.add_put("/upload/resumable/{sid}", self._resume)
        app.router.add_get("/storage/v1/b/{bucket}/o/{name}", self._get)
        app.router.add_delete("/storage/v1/b/{bucket}/o/{name}", self._delete)
        self.start(app)

    def _auth(self, req) -> Optional[web.Response]:
        if self.token and req.headers.get("Authorization") != f"Bearer {self.token}":
            return web.Response(status=401)
        return None

    async def _upload(self, req: web.Request) -> web.Response:
        body = await req.read()
        bad = self._maybe_fail() or self._auth(req)
        if bad is not None:
            return bad
        key = f"{req.match_info['bucket']}/{req.query['name']}"
        if req.query.get("uploadType") == "media":
            self.objects[key] = body
            return web.json_response({"name": req.query["name"]})
        sid = uuid.uuid4().hex
        self.sessions[sid] = {"key": key, "data": bytearray(),
                              "total": int(req.headers.get("X-Upload-Content-Length", -1))}
        return web.Response(headers={"Location": f"{self.url}/upload/resumable/{sid}"})

    async def _resume(self, req: web.Request) -> web.Response:
        body = await req.read()
        bad = self._maybe_fail() or self._auth(req)
        if bad is not None:
            return bad
        s = self.sessions[req.match_info["sid"]]
        cr = req.headers["Content-Range"]
        m = re.match(r"bytes (\d+)-(\d+)/(\d+)", cr)
        if m:
            lo, hi, total = map(int, m.groups())
            if lo != len(s["data"]):
                return web.Response(status=400, text="offset mismatch")
            s["data"] += body
        else:
            total = int(cr.rsplit("/", 1)[1])
        if len(s["data"]) >= total:
            self.objects[s["key"]] = bytes(s["data"])
            return web.json_response({"done": True})
        hdr = {"Range": f"bytes=0-{len(s['data']) - 1}"} if s["data"] else {}
        return web.Response(status=308, headers=hdr)

    async def _get(self, req: web.Request) -> web.Response:
        bad = self._maybe_fail() or self._auth(req)
        if bad is not None:
            return bad
        key = f"{req.match_info['bucket']}/{req.match_info['name']}"
        if key not in self.objects:
            return web.Response(status=404)
        data = self.objects[key]
        rng = req.headers.get("Range")
        if rng:
            lo, hi = map(int, rng.split("=", 1)[1].split("-"))
            return web.Response(status=206, body=data[lo:hi + 1])
        return web.Response(body=data)

    async def _delete(self, req: web.Request) -> web.Response:
        bad = self._auth(req)
        if bad is not None:
            return bad
        self.objects.pop(f"{req.match_info['bucket']}/{req.match_info['name']}", None)
        return web.Response(status=204)


def _main() -> None:
    import sys

    if len(sys.argv) >= 2 and sys.argv[1] == "s3":
        srv = FakeS3Server(*sys.argv[2:4])
        print(f"PORT {srv.port}", flush=True)
        sys.stdin.read()  # until the parent closes our stdin (or exits)
        srv.stop()
    else:
        raise SystemExit("usage: python -m hipsnapshot.storage.fake_servers s3 [key secret]")


if __name__ == "__main__":
    _main()
