"""Google Cloud Storage over the JSON API (aiohttp), with resumable uploads.

Reference: `/root/reference/torchsnapshot/storage_plugins/gcs.py:47-272`
(google-resumable-media + requests in an 8-thread executor, 100 MB chunks,
progress-aware retry deadline).  Neither google-auth nor the GCS SDK exist in
this stack, so this is a direct JSON-API client:

* ``gs://bucket/prefix`` URLs; OAuth2 bearer token from ``storage_options``
  (``token``) or ``GOOGLE_OAUTH_ACCESS_TOKEN``; ``endpoint_url`` overrides
  ``https://storage.googleapis.com`` (the in-process fake in tests);
* uploads: simple media upload below ``chunk_size``, otherwise a resumable
  session (``uploadType=resumable``) sent in ``chunk_size`` pieces
  (multiple of 256 KiB) with ``Content-Range``, resuming from the server's
  committed offset after a transient failure;
* downloads: ``alt=media`` with a ``Range`` header straight into the
  destination buffer, chunked for large ranges;
* ``_RetryStrategy``: one shared deadline per operation, refreshed by any
  progress, exponential backoff with jitter, transient status classifier
  (408/429/5xx) -- the reference's policy, re-implemented.
"""

from __future__ import annotations

import asyncio
import os
import random
import time
from typing import Any, Dict, Optional
from urllib.parse import quote

from ..io_types import ReadIO, StoragePlugin, WriteIO

TRANSIENT = {408, 429, 500, 502, 503, 504}
_CHUNK_ALIGN = 256 * 1024


class GCSError(OSError):
    def __init__(self, msg: str, status: int = 0) -> None:
        super().__init__(msg)
        self.status = status


class _RetryStrategy:
    """Shared deadline refreshed on progress; exponential backoff with jitter."""

    def __init__(self, deadline_s: float = 180.0, base: float = 0.1, cap: float = 8.0) -> None:
        self.deadline_s = deadline_s
        self.base = base
        self.cap = cap
        self.refresh()
        self.attempt = 0

    def refresh(self) -> None:
        self.deadline = time.monotonic() + self.deadline_s
        self.attempt = 0

    def is_transient(self, exc: BaseException) -> bool:
        if isinstance(exc, GCSError):
            return exc.status in TRANSIENT
        return isinstance(exc, (OSError, asyncio.TimeoutError)) and \
            not isinstance(exc, FileNotFoundError)

    async def backoff(self, exc: BaseException) -> None:
        if not self.is_transient(exc) or time.monotonic() >= self.deadline:
            raise exc
        delay = min(self.cap, self.base * (2 ** self.attempt)) * (0.5 + random.random())
        self.attempt += 1
        await asyncio.sleep(min(delay, max(0.0, self.deadline - time.monotonic())))


class GCSStoragePlugin(StoragePlugin):
    def __init__(self, root: str, storage_options: Optional[Dict[str, Any]] = None) -> None:
        opts = dict(storage_options or {})
        components = root.split("/", 1)
        if len(components) != 2 or not components[0]:
            raise RuntimeError("The GCS root path must follow the following pattern: "
                               f"[BUCKET]/[PATH] (got {root})")
        self.bucket, self.prefix = components[0], components[1].strip("/")
        self.token = opts.get("token") or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        self.endpoint = (opts.get("endpoint_url") or "https://storage.googleapis.com").rstrip("/")
        cs = int(opts.get("chunk_size", 100 * 1024 * 1024))
        self.chunk_size = max(_CHUNK_ALIGN, cs // _CHUNK_ALIGN * _CHUNK_ALIGN)
        self.deadline_s = float(opts.get("retry_deadline_s", 180.0))
        self.max_concurrency = int(opts.get("max_concurrency", 16))
        self._session = None
        self._sem: Optional[asyncio.Semaphore] = None

    def _name(self, path: str) -> str:
        return f"{self.prefix}/{path}" if self.prefix else path

    def _headers(self, extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
        h = dict(extra or {})
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    async def _get_session(self):
        if self._session is None or self._session.closed:
            import aiohttp

            self._session = aiohttp.ClientSession(
                connector=aiohttp.TCPConnector(limit=128),
                timeout=aiohttp.ClientTimeout(total=None, sock_read=300))
            self._sem = asyncio.Semaphore(self.max_concurrency)
        return self._session

    async def _call(self, method: str, url: str, expect=(200, 201, 204, 206), **kw):
        sess = await self._get_session()
        async with sess.request(method, url, **kw) as resp:
            data = await resp.read()
            if resp.status in expect:
                return resp.status, dict(resp.headers), data
            if resp.status == 404:
                raise FileNotFoundError(url)
            raise GCSError(f"GCS {method} {url} -> HTTP {resp.status}: {data[:200]!r}",
                           resp.status)

    # -- write --------------------------------------------------------------

    async def write(self, write_io: WriteIO) -> None:
        await self._get_session()
        async with self._sem:
            mv = memoryview(write_io.buf).cast("B")
            name = self._name(write_io.path)
            if mv.nbytes <= self.chunk_size:
                await self._simple_upload(name, mv)
            else:
                await self._resumable_upload(name, mv)

    async def _simple_upload(self, name: str, mv: memoryview) -> None:
        url = (f"{self.endpoint}/upload/storage/v1/b/{self.bucket}/o"
               f"?uploadType=media&name={quote(name, safe='')}")
        retry = _RetryStrategy(self.deadline_s)
        while True:
            try:
                await self._call("POST", url, data=mv.tobytes() if mv.nbytes < (1 << 20) else mv,
                                 headers=self._headers({"Content-Type": "application/octet-stream"}))
                return
            except Exception as e:  # noqa: BLE001
                await retry.backoff(e)

    async def _resumable_upload(self, name: str, mv: memoryview) -> None:
        url = (f"{self.endpoint}/upload/storage/v1/b/{self.bucket}/o"
               f"?uploadType=resumable&name={quote(name, safe='')}")
        retry = _RetryStrategy(self.deadline_s)
        while True:
            try:
                _, hdrs, _ = await self._call(
                    "POST", url, headers=self._headers({"X-Upload-Content-Length": str(mv.nbytes)}))
                session_url = {k.lower(): v for k, v in hdrs.items()}["location"]
                break
            except Exception as e:  # noqa: BLE001
                await retry.backoff(e)
        total = mv.nbytes
        offset = 0
        retry.refresh()
        while offset < total:
            end = min(offset + self.chunk_size, total)
            try:
                status, hdrs, _ = await self._call(
                    "PUT", session_url, expect=(200, 201, 308), data=mv[offset:end],
                    headers=self._headers({"Content-Range": f"bytes {offset}-{end - 1}/{total}"}))
            except Exception as e:  # noqa: BLE001
                await retry.backoff(e)
                # where the service got to: the status query is retried the
                # same way (a flaky service fails it too)
                offset = None
                while offset is None:
                    try:
                        offset = await self._query_offset(session_url, total)
                    except Exception as e2:  # noqa: BLE001
                        await retry.backoff(e2)
                continue
            retry.refresh()  # progress made
            if status in (200, 201):
                return
            rng = {k.lower(): v for k, v in hdrs.items()}.get("range")
            offset = int(rng.rsplit("-", 1)[1]) + 1 if rng else 0

    async def _query_offset(self, session_url: str, total: int) -> int:
        status, hdrs, _ = await self._call("PUT", session_url, expect=(200, 201, 308),
                                           headers=self._headers(
                                               {"Content-Range": f"bytes */{total}"}))
        if status in (200, 201):
            return total
        rng = {k.lower(): v for k, v in hdrs.items()}.get("range")
        return int(rng.rsplit("-", 1)[1]) + 1 if rng else 0

    # -- read / delete ---------------------------------------------------------

    async def read(self, read_io: ReadIO) -> None:
        await self._get_session()
        name = self._name(read_io.path)
        url = f"{self.endpoint}/storage/v1/b/{self.bucket}/o/{quote(name, safe='')}?alt=media"
        async with self._sem:
            if read_io.byte_range is None:
                data = await self._get(url, None)
                if read_io.dest is not None and read_io.dest.nbytes >= len(data):
                    read_io.dest.view[: len(data)] = data
                    read_io.buf = read_io.dest.view[: len(data)]
                else:
                    read_io.buf = memoryview(data)
                return
            lo, hi = read_io.byte_range
            n = hi - lo
            if read_io.dest is not None and read_io.dest.nbytes >= n:
                out = read_io.dest.view[:n]
            else:
                out = memoryview(bytearray(n))
            pos = lo
            while pos < hi:
                end = min(pos + self.chunk_size, hi)
                data = await self._get(url, (pos, end))
                out[pos - lo: pos - lo + len(data)] = data
                pos += len(data)
                if not data:
                    raise GCSError(f"empty range response for {name}")
            read_io.buf = out

    async def _get(self, url: str, rng) -> bytes:
        retry = _RetryStrategy(self.deadline_s)
        headers = self._headers({"Range": f"bytes={rng[0]}-{rng[1] - 1}"} if rng else None)
        while True:
            try:
                _, _, data = await self._call("GET", url, headers=headers)
                return data
            except Exception as e:  # noqa: BLE001
                await retry.backoff(e)

    async def delete(self, path: str) -> None:
        name = self._name(path)
        url = f"{self.endpoint}/storage/v1/b/{self.bucket}/o/{quote(name, safe='')}"
        retry = _RetryStrategy(self.deadline_s)
        while True:
            try:
                await self._call("DELETE", url, headers=self._headers())
                return
            except Exception as e:  # noqa: BLE001
                await retry.backoff(e)

    async def close(self) -> None:
        if self._session is not None and not self._session.closed:
            await self._session.close()
        self._session = None
