"""In-process fake S3 and GCS servers (aiohttp.web) for tests and benchmarks.

There is no network on the build or GPU boxes, so the S3/GCS plugins are
exercised end to end against these: the fake S3 server VERIFIES every SigV4
signature (recomputed from the raw request with the shared secret) and
implements PUT/GET(Range)/DELETE, multipart uploads and ListObjectsV2; the
fake GCS server implements media + resumable uploads (308 / Range protocol),
ranged ``alt=media`` downloads and DELETE.  Both support fault injection
(``fail_next(n, status)``) to test the retry paths.
"""

from __future__ import annotations

import asyncio
import datetime as _dt
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

    def fail_next(self, n: int = 1, status: int = 503) -> None:
        self.fail_queue.extend([status] * n)

    def _maybe_fail(self) -> Optional[web.Response]:
        self.requests += 1
        if self.fail_queue:
            return web.Response(status=self.fail_queue.pop(0), text="injected")
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


class FakeS3Server(_ServerThread):
    def __init__(self, access_key: str = "AKIDFAKE", secret: str = "fake-secret",
                 region: str = "us-east-1") -> None:
        super().__init__()
        self.access_key, self.secret, self.region = access_key, secret, region
        self.objects: Dict[str, bytes] = {}
        self.uploads: Dict[str, Dict[int, bytes]] = {}
        app = web.Application(client_max_size=1 << 40)
        app.router.add_route("*", "/{bucket}", self._bucket)
        app.router.add_route("*", "/{bucket}/{key:.*}", self._object)
        self.start(app)

    def _verify(self, req: web.Request, body: bytes) -> Optional[web.Response]:
        auth = req.headers.get("Authorization", "")
        m = re.match(r"AWS4-HMAC-SHA256 Credential=([^/]+)/(\d{8})/([^/]+)/s3/aws4_request, "
                     r"SignedHeaders=([^,]+), Signature=([0-9a-f]{64})$", auth)
        if not m or m.group(1) != self.access_key:
            return web.Response(status=403, text=f"bad auth header {auth!r}")
        signed = m.group(4).split(";")
        hdrs = {h: req.headers.get(h, "") for h in signed
                if h not in ("host", "x-amz-date", "x-amz-content-sha256")}
        now = _dt.datetime.strptime(req.headers["x-amz-date"], "%Y%m%dT%H%M%SZ").replace(
            tzinfo=_dt.timezone.utc)
        query = {k: v for k, v in req.query.items()}
        expect = sigv4_headers(req.method, req.headers["Host"], req.path, query, hdrs,
                               req.headers["x-amz-content-sha256"], self.access_key,
                               self.secret, m.group(3), now=now,
                               session_token=req.headers.get("x-amz-security-token"))
        if expect["Authorization"] != auth:
            return web.Response(status=403, text="SignatureDoesNotMatch")
        ph = req.headers["x-amz-content-sha256"]
        if ph not in ("UNSIGNED-PAYLOAD",):
            import hashlib

            if hashlib.sha256(body).hexdigest() != ph:
                return web.Response(status=400, text="XAmzContentSHA256Mismatch")
        return None

    async def _bucket(self, req: web.Request) -> web.Response:
        body = await req.read()
        bad = self._maybe_fail() or self._verify(req, body)
        if bad is not None:
            return bad
        bucket = req.match_info["bucket"]
        if req.method == "GET" and req.query.get("list-type") == "2":
            prefix = req.query.get("prefix", "")
            keys = sorted(k.split("/", 1)[1] for k in self.objects
                          if k.startswith(f"{bucket}/{prefix}"))
            xml = "<ListBucketResult>" + "".join(f"<Contents><Key>{k}</Key></Contents>"
                                                 for k in keys) + "</ListBucketResult>"
            return web.Response(text=xml, content_type="application/xml")
        return web.Response(status=400)

    async def _object(self, req: web.Request) -> web.Response:
        body = await req.read()
        bad = self._maybe_fail() or self._verify(req, body)
        if bad is not None:
            return bad
        key = f"{req.match_info['bucket']}/{req.match_info['key']}"
        q = req.query
        if req.method == "POST" and "uploads" in q:
            uid = uuid.uuid4().hex
            self.uploads[uid] = {}
            return web.Response(text=f"<InitiateMultipartUploadResult><UploadId>{uid}</UploadId>"
                                     "</InitiateMultipartUploadResult>",
                                content_type="application/xml")
        if req.method == "PUT" and "uploadId" in q:
            self.uploads[q["uploadId"]][int(q["partNumber"])] = body
            return web.Response(headers={"ETag": f'"{q["partNumber"]}-{len(body)}"'})
        if req.method == "POST" and "uploadId" in q:
            parts = self.uploads.pop(q["uploadId"])
            nums = [int(n) for n in re.findall(r"<PartNumber>(\d+)</PartNumber>", body.decode())]
            self.objects[key] = b"".join(parts[n] for n in nums)
            return web.Response(text="<CompleteMultipartUploadResult/>",
                                content_type="application/xml")
        if req.method == "DELETE" and "uploadId" in q:
            self.uploads.pop(q["uploadId"], None)
            return web.Response(status=204)
        if req.method == "PUT":
            self.objects[key] = body
            return web.Response(headers={"ETag": '"x"'})
        if req.method == "GET":
            if key not in self.objects:
                return web.Response(status=404, text="NoSuchKey")
            data = self.objects[key]
            rng = req.headers.get("Range")
            if rng:
                lo, hi = map(int, rng.split("=", 1)[1].split("-"))
                return web.Response(status=206, body=data[lo:hi + 1])
            return web.Response(body=data)
        if req.method == "DELETE":
            self.objects.pop(key, None)
            return web.Response(status=204)
        return web.Response(status=405)


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
