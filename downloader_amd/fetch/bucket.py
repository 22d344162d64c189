"""``bucket://`` source (reference ``methods.bucket``, lib/download.js:199-227).

Grammar: ``bucket://<endpoint>,<bucket>,<accessKey>,<secretKey>,<subFolder>`` - split on ``,``,
TLS always on (reference ``useSSL: true``; ``download.bucket_secure`` may turn it off for
local tests). Objects under ``subFolder/`` are listed recursively and each is written to
``path.join(dir, name.replace(subFolder, ''))`` (JS ``String.replace`` with a string replaces the
first occurrence only). The reference fetches objects one by one; here up to
``bucket_concurrency`` run at once. Credentials are redacted in logs (App. A #19).
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass
from typing import List, Optional

from ..models.keys import node_join
from ..stages.jobdir import inside
from ..utils.aio import gather_strict
from ..utils.log import Logger, NullLogger


@dataclass
class BucketSource:
    endpoint: str
    bucket: str
    access_key: str
    secret_key: str
    sub_folder: str

    def redacted(self) -> str:
        return f"bucket://{self.endpoint},{self.bucket},{self.access_key},***,{self.sub_folder}"


def parse_bucket_uri(uri: str) -> BucketSource:
    params = uri.split(",")
    if len(params) < 5:
        raise ValueError("bucket:// URI must be bucket://endpoint,bucket,accessKey,secretKey,subFolder")
    endpoint = params[0].replace("bucket://", "", 1)
    return BucketSource(endpoint, params[1], params[2], params[3], params[4])


def local_name(download_dir: str, item_name: str, sub_folder: str) -> str:
    return node_join(download_dir, item_name.replace(sub_folder, "", 1))


async def fetch_bucket(uri: str, download_dir: str, secure: bool = True, concurrency: int = 4,
                       transports=None, logger: Optional[Logger] = None, progress=None,
                       native: bool = True, ssl_verify: bool = True,
                       ca_file: str = "", native_tls: bool = True) -> List[str]:
    from ..s3.client import S3Client
    log = logger or NullLogger()
    src = parse_bucket_uri(uri)
    log.info("bucket", src.redacted())
    log.info("bucket", f"using s3 endpoint: {src.endpoint}")
    client = S3Client(src.endpoint, src.access_key, src.secret_key, secure=secure,
                      transports=transports, native=native, ssl_verify=ssl_verify,
                      ca_file=ca_file, native_tls=native_tls)
    try:
        prefix = src.sub_folder.rstrip("/") + "/"
        items = await client.list_objects(src.bucket, prefix, recursive=True)
        sem = asyncio.Semaphore(max(1, concurrency))
        out: List[str] = []

        async def one(name: str) -> None:
            dst = local_name(download_dir, name, src.sub_folder)
            if not inside(download_dir, dst):   # '../job2/x' must not reach a sibling dir
                raise ValueError(f"object {name!r} escapes the download directory")
            async with sem:
                log.info(f"Downloading file '{name}' from bucket '{src.bucket}' to '{dst}'")
                await client.fget_object(src.bucket, name, dst, progress=progress)
            out.append(dst)

        await gather_strict(*(one(it.name) for it in items if it.name and not it.name.endswith("/")))
        return out
    finally:
        await client.close()
