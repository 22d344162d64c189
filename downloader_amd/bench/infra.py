"""Bench infrastructure: launches the native ``blobd`` peer (HTTP origin + S3 sink)."""
from __future__ import annotations

import json
import os
import subprocess
import tempfile
import time
import urllib.request
from pathlib import Path
from typing import Dict, Optional, Tuple

from ..ops import build

PKG = Path(__file__).resolve().parents[1]


def self_signed_cert(directory: str, name: str = "127.0.0.1") -> Tuple[str, str]:
    """Throwaway certificate + key for the TLS bench (openssl CLI; SAN = the IP / name)."""
    crt, key = os.path.join(directory, "blobd.crt"), os.path.join(directory, "blobd.key")
    san = f"IP:{name}" if name.replace(".", "").isdigit() else f"DNS:{name}"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", crt, "-days", "2", "-subj", f"/CN={name}", "-addext",
                    f"subjectAltName={san}"], check=True, capture_output=True, timeout=120)
    return crt, key


class Blobd:
    def __init__(self, keep_bytes: int = 1 << 20, default_size: int = 100_000_000,
                 host: str = "127.0.0.1", files_root: str = "", sink: str = "checksum",
                 tls: Optional[Tuple[str, str]] = None, s3_fail_rate: float = 0.0,
                 synth_bucket: str = "", synth_objects: Optional[Dict[str, int]] = None,
                 s3_corrupt_rate: float = 0.0,
                 synth_files: Optional[Dict[str, Tuple[int, int]]] = None,
                 crc_check: int = 1, crc_salt: int = 0, synth_shift: int = 0):
        self.files_root = files_root
        # webseed files served from the origin pool: relpath -> (size, seed)
        self.synth_files = dict(synth_files or {})
        self.tls = tls                  # (cert PEM, key PEM): serve https
        self.s3_fail_rate = s3_fail_rate  # share of object/part PUTs answered 503 SlowDown
        # share of checksummed PUT bodies with one byte flipped on arrival (-> 400 BadDigest)
        self.s3_corrupt_rate = s3_corrupt_rate
        self.synth_bucket = synth_bucket  # read-only source bucket of synthetic objects
        self.synth_objects = dict(synth_objects or {})
        self.sink = sink
        # recompute the CRC32C of 1 in crc_check checksummed bodies (salted hash of key + part:
        # fixed for a run, unknown to the sender; 0 salt = random); the rest are dropped in the
        # kernel after their trailer is checked for form
        self.crc_check = max(1, int(crc_check))
        self.crc_salt = int(crc_salt)
        self.synth_shift = int(synth_shift)   # serve the synth files this many bytes off (tests)
        self.keep_bytes = keep_bytes
        self.default_size = default_size
        self.host = host
        self.proc: Optional[subprocess.Popen] = None
        self.port = 0

    def start(self, timeout: float = 30.0) -> "Blobd":
        # STAGER_BLOBD_EXE: another build of the peer (A/B of a generator change)
        exe = os.environ.get("STAGER_BLOBD_EXE") or build.build_blobd(verbose=False)
        d = tempfile.mkdtemp(prefix="blobd-")
        pf = os.path.join(d, "port")
        self.proc = subprocess.Popen(
            [str(exe), "--host", self.host, "--port", "0", "--port-file", pf,
             "--keep-bytes", str(self.keep_bytes), "--default-size", str(self.default_size)]
            + (["--files-root", self.files_root] if self.files_root else [])
            + ["--sink", self.sink]
            + (["--crc-check", str(self.crc_check)] if self.crc_check > 1 else [])
            + (["--crc-salt", str(self.crc_salt)] if self.crc_salt else [])
            + (["--synth-shift", str(self.synth_shift)] if self.synth_shift else [])
            # the sink's kernel drops wake per 256 KiB, not per segment (STAGER_BLOBD_RCVLOWAT_KB:
            # another mark, 0 = off; profiles/r6/check2/lowat*)
            + (["--rcvlowat", os.environ.get("STAGER_BLOBD_RCVLOWAT_KB", "256")]
               if os.environ.get("STAGER_BLOBD_RCVLOWAT_KB", "256") != "0" else [])
            + (["--tls-cert", self.tls[0], "--tls-key", self.tls[1]] if self.tls else [])
            + (["--s3-fail-rate", str(self.s3_fail_rate)] if self.s3_fail_rate else [])
            + (["--s3-corrupt-rate", str(self.s3_corrupt_rate)] if self.s3_corrupt_rate else [])
            + (["--synth-bucket", self.synth_bucket, "--synth-manifest",
                self._manifest(d)] if self.synth_bucket else [])
            + (["--synth-files", self._files_manifest(d)] if self.synth_files else []),
            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        t0 = time.time()
        while not os.path.exists(pf):
            if self.proc.poll() is not None:
                raise RuntimeError(f"blobd exited: {self.proc.stderr.read().decode()}")
            if time.time() - t0 > timeout:
                self.stop()
                raise RuntimeError("blobd did not start")
            time.sleep(0.02)
        self.port = int(open(pf).read().strip())
        return self

    @property
    def endpoint(self) -> str:
        return f"{self.host}:{self.port}"

    def _manifest(self, d: str) -> str:
        p = os.path.join(d, "synth-manifest")
        with open(p, "w") as f:
            for k, n in self.synth_objects.items():
                f.write(f"{k} {n}\n")
        return p

    def _files_manifest(self, d: str) -> str:
        p = os.path.join(d, "synth-files")
        with open(p, "w") as f:
            for rel, (n, seed) in self.synth_files.items():
                f.write(f"{rel} {n} {seed}\n")
        return p

    def pool(self) -> bytes:
        """The origin's byte pool (64 MiB + 4 KiB): synthetic byte o of seed s =
        pool[(o + 7919 s) % len(pool)]."""
        with urllib.request.urlopen(f"http://{self.endpoint}/_pool", timeout=60) as r:
            return r.read()

    @property
    def scheme(self) -> str:
        return "https" if self.tls else "http"

    def media_url(self, name: str, size: int, seed: int) -> str:
        return f"{self.scheme}://{self.endpoint}/media/{name}?size={size}&seed={seed}"

    def files_url(self, rel: str = "") -> str:
        return f"{self.scheme}://{self.endpoint}/files/{rel}"

    def cpu_seconds(self) -> float:
        """user+sys CPU time of the blobd process (from /proc/<pid>/stat)."""
        if self.proc is None:
            return 0.0
        try:
            with open(f"/proc/{self.proc.pid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError):
            return 0.0

    def crc_selected(self, key: str, part: int = 0) -> bool:
        """Does the sink recompute the CRC32C of this body (``--crc-check`` subset)?"""
        from urllib.parse import urlencode
        with urllib.request.urlopen(f"http://{self.endpoint}/_crc_selected?"
                                    + urlencode({"key": key, "part": part}), timeout=10) as r:
            return r.read().strip() == b"1"

    def stats(self) -> Dict[str, int]:
        ctx = None
        if self.tls:
            import ssl
            ctx = ssl.create_default_context(cafile=self.tls[0])
        with urllib.request.urlopen(f"{self.scheme}://{self.endpoint}/_stats", timeout=10,
                                    context=ctx) as r:
            return json.loads(r.read())

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
        self.proc = None

    def __enter__(self) -> "Blobd":
        return self.start()

    def __exit__(self, *a) -> None:
        self.stop()
