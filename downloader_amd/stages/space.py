"""Free-space check before a job writes its payload to the staging filesystem.

The reference streams into ``<download_path>/<id>`` until the disk fills, then fails with
ENOSPC mid-transfer (after fetching most of the bytes) and leaves the partial data behind.
Here the HTTP disk path (once the origin reported the size) and the torrent disk path (once
the metadata is known) first compare what is still to be written - file sizes minus what is
already allocated, so a resumed job only needs the rest - plus ``download.min_free_bytes``
with the filesystem's free space, and fail fast with ENOSPC. Stream staging writes nothing
locally and is not checked.
"""
from __future__ import annotations

import errno
import os
import shutil
from typing import Iterable, Tuple


class InsufficientSpace(OSError):
    def __init__(self, path: str, need: int, free: int, reserve: int):
        super().__init__(errno.ENOSPC, f"not enough space under {path}: {need} B still to "
                                       f"write + {reserve} B reserve, {free} B free")
        self.need, self.free, self.reserve = need, free, reserve


def allocated(path: str) -> int:
    """Bytes already on disk for ``path`` (allocated blocks: a sparse, pre-sized file counts
    only what was written)."""
    try:
        st = os.stat(path)
    except OSError:
        return 0
    return min(st.st_size, st.st_blocks * 512)


def still_to_write(files: Iterable[Tuple[str, int]]) -> int:
    return sum(max(0, n - allocated(p)) for p, n in files)


def ensure_space(dirpath: str, need: int, reserve: int = 0) -> None:
    if need <= 0 and reserve <= 0:
        return
    probe = dirpath
    while probe and not os.path.isdir(probe):        # job dir may not exist yet
        probe = os.path.dirname(probe)
    free = shutil.disk_usage(probe or ".").free
    if need + reserve > free:
        raise InsufficientSpace(dirpath, need, free, reserve)
