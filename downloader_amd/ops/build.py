"""In-tree build of the native pieces (no JIT cache: the .so files travel with the repo).

Targets
  * ``_native``   host C++17 pybind11 module: OpenSSL EVP hashing + zero-copy HTTP transport
  * ``_gpuhash``  HIP/gfx950 pybind11 module: batched SHA-1 piece verification on the MI355X
  * ``blobd``     C++ multi-threaded HTTP origin + S3 sink used by the bench harness

Run ``python -m downloader_amd.ops.build`` (``__graft_entry__.build()`` calls it).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List, Sequence

PKG = Path(__file__).resolve().parents[1]
CSRC = PKG / "csrc"
OPS = PKG / "ops"
BIN = PKG / "bin"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _pybind_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _stale(out: Path, srcs: Sequence[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(s.stat().st_mtime > t for s in srcs)


def _run(cmd: List[str], verbose: bool) -> None:
    """Run a compile whose last two arguments are ``-o <out>``: the compiler writes a private
    temporary file that then atomically replaces ``out``, so concurrent builders (the ranks of
    a multi-GPU bench finding a stale blobd at the same moment) never leave a truncated file
    and a running binary is never overwritten in place."""
    assert cmd[-2] == "-o", cmd
    out = cmd[-1]
    tmp = f"{out}.tmp.{os.getpid()}"
    cmd = cmd[:-1] + [tmp]
    if verbose:
        print("+", " ".join(cmd[:-1] + [out]), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd[:3])} ... (exit {r.returncode})")
    os.replace(tmp, out)


def build_native(force: bool = False, verbose: bool = True) -> Path:
    srcs = [CSRC / "module.cpp", CSRC / "hashing.cpp", CSRC / "sha1_mb.cpp", CSRC / "transfer.cpp",
            CSRC / "tls.cpp", CSRC / "peerwire.cpp"]
    out = OPS / f"_native{EXT}"
    if force or _stale(out, srcs + [CSRC / "native.h", CSRC / "crc32c.h",
                                    CSRC / "gpu_part_api.h"]):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
               "-march=x86-64-v3", "-Wall", "-Wno-unused-result",
               *_pybind_includes(), *[str(s) for s in srcs], "-lssl", "-lcrypto", "-lpthread",
               "-o", str(out)]
        _run(cmd, verbose)
    return out


def build_gpuhash(force: bool = False, verbose: bool = True) -> Path:
    srcs = [CSRC / "gpu_sha1.hip"]
    out = OPS / f"_gpuhash{EXT}"
    if force or _stale(out, srcs + [CSRC / "gpu_part_api.h", CSRC / "part_dispatch.h"]):
        hipcc = str(ROCM / "bin" / "hipcc")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
               "-fvisibility=hidden", *_pybind_includes(), str(srcs[0]), "-o", str(out)]
        _run(cmd, verbose)
    return out


def build_blobd(force: bool = False, verbose: bool = True) -> Path:
    srcs = [CSRC / "blobd.cpp"]
    BIN.mkdir(exist_ok=True)
    out = BIN / "blobd"
    if force or _stale(out, srcs + [CSRC / "crc32c.h"]):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O3", "-std=c++17", "-march=x86-64-v3", "-Wall", str(srcs[0]),
               "-lssl", "-lcrypto", "-lpthread", "-o", str(out)]
        _run(cmd, verbose)
    return out


def build_swarmd(force: bool = False, verbose: bool = True) -> Path:
    """Heterogeneous fake seeders for the swarm bench / tests (csrc/swarmd.cpp)."""
    srcs = [CSRC / "swarmd.cpp"]
    BIN.mkdir(exist_ok=True)
    out = BIN / "swarmd"
    if force or _stale(out, srcs):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O2", "-std=c++17", "-Wall", str(srcs[0]), "-lpthread", "-o", str(out)]
        _run(cmd, verbose)
    return out


def build_relaybench(force: bool = False, verbose: bool = True) -> Path:
    """Per-byte CPU of the relay modes (csrc/relaybench.cpp): the copy / CRC floor."""
    srcs = [CSRC / "relaybench.cpp"]
    BIN.mkdir(exist_ok=True)
    out = BIN / "relaybench"
    if force or _stale(out, srcs + [CSRC / "crc32c.h"]):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O3", "-std=c++17", "-march=x86-64-v3", "-Wall", str(srcs[0]),
               "-lpthread", "-o", str(out)]
        _run(cmd, verbose)
    return out


SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
              "tsan": ["-fsanitize=thread"]}


def build_selftest(kind: str, force: bool = False, verbose: bool = True) -> Path:
    """Host-only sanitizer build of the native code's self-test."""
    srcs = [CSRC / "selftest.cpp", CSRC / "hashing.cpp", CSRC / "sha1_mb.cpp", CSRC / "transfer.cpp",
            CSRC / "tls.cpp", CSRC / "peerwire.cpp"]
    BIN.mkdir(exist_ok=True)
    out = BIN / f"selftest_{kind}"
    if force or _stale(out, srcs + [CSRC / "native.h", CSRC / "crc32c.h",
                                    CSRC / "gpu_part_api.h", CSRC / "part_dispatch.h"]):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O1", "-g", "-std=c++17", "-msse4.2", *SANITIZERS[kind],
               *[str(s) for s in srcs],
               "-lssl", "-lcrypto", "-lpthread", "-o", str(out)]
        _run(cmd, verbose)
    return out


def build_all(force: bool = False, verbose: bool = True, gpu: bool = True) -> None:
    build_native(force, verbose)
    if (CSRC / "blobd.cpp").exists():
        build_blobd(force, verbose)
    if (CSRC / "relaybench.cpp").exists():
        build_relaybench(force, verbose)
    if (CSRC / "swarmd.cpp").exists():
        build_swarmd(force, verbose)
    if gpu and (CSRC / "gpu_sha1.hip").exists():
        if not (ROCM / "bin" / "hipcc").exists():
            raise RuntimeError("hipcc not found; cannot build the gfx950 kernels")
        build_gpuhash(force, verbose)


def clean() -> None:
    for p in OPS.glob("_*.so"):
        p.unlink()
    if BIN.exists():
        shutil.rmtree(BIN)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
