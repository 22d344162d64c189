"""Media-file selector (reference lib/process.js:29-99).

Walk semantics reproduce klaw@3 as driven by the reference: the root is visited first and
skipped (it is a directory); each directory's entries are read in sorted byte order (libuv
``scandir`` + ``alphasort``), every *child* path is passed through the filter, survivors are
pushed onto a stack in reverse, so the output is depth-first lexicographic and a rejected
directory is never descended into.

Per child (evaluated in order):

===== ===================================================================== ======
dir   the root has exactly one entry and it is this dir                       keep
dir   ``media.type == MOVIE``                                                  keep
dir   ``/\\/extras|\\/commentary/i`` matches the path                            drop
dir   ``/s\\d+|season/i`` matches the basename                                  keep
dir   otherwise                                                               drop
file  ``extname(name)`` in {.mp4,.mkv,.mov,.webm} (case-sensitive by default)  keep
===== ===================================================================== ======

Deliberate fixes (flag-gated back to the reference behaviour):
  * #14 the extras/commentary regex is tested on the path *relative to the job root*
    (the reference tests the absolute path, so a ``download_path`` containing ``/extras``
    would reject every directory).
  * #16 the "sole top-level directory" rule applies only at depth 1.
  * symlink loops are cut (klaw follows symlinks without a visited set).
"""
from __future__ import annotations

import os
import re
import stat as _stat
from typing import Iterable, List, Optional, Sequence

from ..models import api
from ..utils.log import Logger, NullLogger

DEFAULT_MEDIA_EXTS = (".mp4", ".mkv", ".mov", ".webm")
_EXTRAS = re.compile(r"/extras|/commentary", re.IGNORECASE)
_SEASON = re.compile(r"s\d+|season", re.IGNORECASE)


class NoMediaFilesError(Exception):
    """Raised by the process stage when the walk keeps nothing (lib/process.js:109-111)."""

    def __init__(self) -> None:
        super().__init__("Failed to find any suitable media files")


def node_extname(path: str) -> str:
    """Node's POSIX ``path.extname`` (same scan: ``.mkv`` -> '', ``a.`` -> '.', ``..md`` -> '.md')."""
    start_dot = -1
    start_part = 0
    end = -1
    matched_slash = True
    pre_dot_state = 0
    for i in range(len(path) - 1, -1, -1):
        c = path[i]
        if c == "/":
            if not matched_slash:
                start_part = i + 1
                break
            continue
        if end == -1:
            matched_slash = False
            end = i + 1
        if c == ".":
            if start_dot == -1:
                start_dot = i
            elif pre_dot_state != 1:
                pre_dot_state = 1
        elif start_dot != -1:
            pre_dot_state = -1
    if (start_dot == -1 or end == -1 or pre_dot_state == 0
            or (pre_dot_state == 1 and start_dot == end - 1 and start_dot == start_part + 1)):
        return ""
    return path[start_dot:end]


def _sorted_entries(path: str) -> List[str]:
    # libuv sorts scandir results with strcmp on the raw bytes.
    names = os.listdir(os.fsencode(path))
    names.sort()
    return [os.fsdecode(n) for n in names]


class MediaSelector:
    def __init__(self, media_exts: Sequence[str] = DEFAULT_MEDIA_EXTS,
                 case_insensitive_exts: bool = False, legacy_full_path_extras: bool = False,
                 legacy_any_depth_sole_dir: bool = False, logger: Optional[Logger] = None):
        self.case_insensitive = case_insensitive_exts
        self.exts = {e.lower() for e in media_exts} if case_insensitive_exts else set(media_exts)
        self.legacy_full_path_extras = legacy_full_path_extras
        self.legacy_any_depth_sole_dir = legacy_any_depth_sole_dir
        self.log = logger or NullLogger()

    def _is_media(self, name: str) -> bool:
        ext = node_extname(name)
        if self.case_insensitive:
            ext = ext.lower()
        return ext in self.exts

    def _keep(self, root: str, root_entries: List[str], item: str, is_dir: bool, depth: int,
              movie: bool) -> bool:
        name = os.path.basename(item)
        if not is_dir:
            return self._is_media(name)
        if (depth == 1 or self.legacy_any_depth_sole_dir) and len(root_entries) == 1 \
                and root_entries[0] == name:
            self.log.info(f"{item} is allowed because its the only top level directory")
            return True
        if movie:
            return True
        probe = item if self.legacy_full_path_extras else "/" + os.path.relpath(item, root)
        if _EXTRAS.search(probe):
            return False
        return bool(_SEASON.search(name))

    def find(self, root: str, media_type: int) -> List[str]:
        root = os.path.abspath(root)
        movie = media_type == api.string_to_enum("MediaType", "MOVIE")
        root_entries = _sorted_entries(root)
        files: List[str] = []
        seen = set()
        # stack of (path, depth); the root is visited first and skipped (directory).
        stack = [(root, 0)]
        while stack:
            path, depth = stack.pop()
            try:
                st = os.stat(path)
            except FileNotFoundError:
                continue
            if not _stat.S_ISDIR(st.st_mode):
                files.append(path)
                continue
            key = (st.st_dev, st.st_ino)
            if key in seen:
                continue
            seen.add(key)
            entries = root_entries if depth == 0 else _sorted_entries(path)
            keep: List[tuple] = []
            for name in entries:
                child = os.path.join(path, name)
                try:
                    is_dir = os.path.isdir(child)
                except OSError:
                    continue
                ok = self._keep(root, root_entries, child, is_dir, depth + 1, movie)
                rel = os.path.relpath(child, root)
                kind = "directory" if is_dir else "file"
                if ok:
                    self.log.info(f"including {kind} '{rel}'")
                    keep.append((child, depth + 1))
                else:
                    self.log.warn(f"skipping {kind} '{rel}'")
            stack.extend(reversed(keep))
        return files

    def accepts_single_file(self, filename: str) -> bool:
        """Whether a lone top-level file with this name would be selected (stream fast path)."""
        return self._is_media(filename)

    def find_virtual(self, root: str, rel_files: Sequence[str], media_type: int) -> List[str]:
        """The same walk over a tree that does not exist yet - e.g. the file list of a torrent
        before its data arrives - given as paths relative to ``root``. Returns the absolute
        paths ``find(root, ...)`` will return once exactly those files are on disk."""
        root = os.path.abspath(root)
        movie = media_type == api.string_to_enum("MediaType", "MOVIE")
        tree: dict = {}
        for rel in rel_files:
            node = tree
            parts = [p for p in rel.split("/") if p]
            for d in parts[:-1]:
                node = node.setdefault(d, {})
                if node is None:
                    break
            if parts:
                node.setdefault(parts[-1], None)

        def entries(node: dict) -> List[str]:
            return sorted(node, key=os.fsencode)

        root_entries = entries(tree)
        files: List[str] = []
        stack = [(root, tree, 0)]
        while stack:
            path, node, depth = stack.pop()
            if node is None:
                files.append(path)
                continue
            keep = []
            for name in (root_entries if depth == 0 else entries(node)):
                child = os.path.join(path, name)
                sub = node[name]
                if self._keep(root, root_entries, child, sub is not None, depth + 1, movie):
                    keep.append((child, sub, depth + 1))
            stack.extend(reversed(keep))
        return files


def find_media_files(root: str, media_type: int, logger: Optional[Logger] = None,
                     **kw) -> List[str]:
    """``findMediaFiles(absPath, media, logger)`` (lib/process.js:29)."""
    return MediaSelector(logger=logger, **kw).find(root, media_type)


def select_from_config(cfg, logger: Optional[Logger] = None) -> MediaSelector:
    p = cfg.process
    return MediaSelector(p.media_exts, p.case_insensitive_exts, p.legacy_full_path_extras,
                         p.legacy_any_depth_sole_dir, logger)


__all__: Iterable[str] = ["MediaSelector", "find_media_files", "NoMediaFilesError",
                          "node_extname", "select_from_config"]
