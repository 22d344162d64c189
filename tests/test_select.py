"""Media selector - golden cases ported from the reference's only unit tests
(test/process/filter_dirs.js:17-82) plus the App. B truth table and property tests.

The reference fixture trees hold zero-byte ``.mkv`` files; the same trees are recreated here.
"""
from __future__ import annotations

import os

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from downloader_amd.models import api
from downloader_amd.stages.select import MediaSelector, find_media_files, node_extname
from downloader_amd.utils.log import NullLogger, make_test_logger

TV = api.string_to_enum("MediaType", "TV")
MOVIE = api.string_to_enum("MediaType", "MOVIE")
LOG = make_test_logger("process")  # USE_REAL_LOGGER=1 shows the selector's decisions


def make_tree(root, files):
    for rel in files:
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        open(p, "wb").close()
    return str(root)


def test_should_filter_non_season_directories(tmp_path):
    # reference: test/process/filter_dirs.js:21-41
    root = make_tree(tmp_path / "should_filter_non_season_directories", [
        "Season 1/KonoSuba S1E1.mkv", "Extras/KonoSuba OVA.mkv",
        "Commentary/KonoSuba Season 1 Commentary.mkv", "S1/KonoSuba S1E1.mkv"])
    files = find_media_files(root, TV, LOG)
    assert len(files) == 2
    assert files[0] == os.path.join(root, "S1/KonoSuba S1E1.mkv")
    assert files[1] == os.path.join(root, "Season 1/KonoSuba S1E1.mkv")


def test_should_read_all_dirs_when_processing_a_movie(tmp_path):
    # reference: test/process/filter_dirs.js:43-61
    root = make_tree(tmp_path / "movie", ["Some Movie Dir/Your Name.mkv"])
    files = find_media_files(root, MOVIE, LOG)
    assert files == [os.path.join(root, "Some Movie Dir/Your Name.mkv")]


def test_should_read_with_top_level_dir(tmp_path):
    # reference: test/process/filter_dirs.js:63-81 ("should real with top level dir")
    root = make_tree(tmp_path / "top", ["Some Movie Dir/Your Name.mkv"])
    files = find_media_files(root, TV, LOG)
    assert files == [os.path.join(root, "Some Movie Dir/Your Name.mkv")]


def test_movie_keeps_extras(tmp_path):
    root = make_tree(tmp_path / "m", ["Extras/a.mkv", "Main/b.mp4", "c.webm", "d.txt"])
    files = [os.path.relpath(f, root) for f in find_media_files(root, MOVIE, LOG)]
    assert files == ["Extras/a.mkv", "Main/b.mp4", "c.webm"]


def test_tv_season_regex_is_unanchored(tmp_path):
    # App. B: /s\d+|season/i matches "Videos2" (s2) but not "Specials"
    root = make_tree(tmp_path / "t", ["Videos2/a.mkv", "Specials/b.mkv", "x.mov"])
    files = [os.path.relpath(f, root) for f in find_media_files(root, TV, LOG)]
    assert files == ["Videos2/a.mkv", "x.mov"]


def test_extension_case_sensitive_by_default(tmp_path):
    root = make_tree(tmp_path / "c", ["A.MKV", "b.mkv"])
    assert [os.path.basename(f) for f in find_media_files(root, MOVIE, LOG)] == ["b.mkv"]
    sel = MediaSelector(case_insensitive_exts=True)
    assert [os.path.basename(f) for f in sel.find(root, MOVIE)] == ["A.MKV", "b.mkv"]


def test_depth_first_lexicographic_order(tmp_path):
    root = make_tree(tmp_path / "o", ["b/2.mkv", "b/1.mkv", "a/z.mkv", "a/S01/e.mkv", "0.mkv"])
    files = [os.path.relpath(f, root) for f in find_media_files(root, MOVIE, LOG)]
    assert files == ["0.mkv", "a/S01/e.mkv", "a/z.mkv", "b/1.mkv", "b/2.mkv"]


def test_download_path_containing_extras_is_not_poisoned(tmp_path):
    # App. A #14: reference tests the absolute path; we test the job-relative path.
    root = make_tree(tmp_path / "extras-store" / "job", ["Season 1/a.mkv", "Other/b.mkv"])
    files = [os.path.relpath(f, root) for f in find_media_files(root, TV, LOG)]
    assert files == ["Season 1/a.mkv"]
    legacy = MediaSelector(legacy_full_path_extras=True).find(root, TV)
    assert legacy == []


def test_sole_dir_rule_depth_one_only(tmp_path):
    # App. A #16: nested dir with the same name as the sole root entry is not auto-kept.
    root = make_tree(tmp_path / "s", ["Show/Show/a.mkv", "Show/b.mkv"])
    files = [os.path.relpath(f, root) for f in find_media_files(root, TV, LOG)]
    assert files == ["Show/b.mkv"]
    legacy = MediaSelector(legacy_any_depth_sole_dir=True).find(root, TV)
    assert [os.path.relpath(f, root) for f in legacy] == ["Show/Show/a.mkv", "Show/b.mkv"]


def test_symlink_loop_terminates(tmp_path):
    root = make_tree(tmp_path / "l", ["S1/a.mkv"])
    os.symlink(os.path.join(root, "S1"), os.path.join(root, "S1", "S1loop"))
    files = [os.path.relpath(f, root) for f in find_media_files(root, TV, LOG)]
    assert files[0] == "S1/a.mkv"
    assert files == ["S1/a.mkv"]  # the symlinked dir is the same inode: cut


@pytest.mark.parametrize("name,ext", [
    ("index.html", ".html"), ("index.coffee.md", ".md"), ("index.", "."), ("index", ""),
    (".index", ""), (".index.md", ".md"), ("..", ""), ("..md", ".md"), ("a.b.mkv", ".mkv"),
    (".mkv", ""), ("x.torrent", ".torrent"),
])
def test_node_extname(name, ext):
    assert node_extname(name) == ext


_seg = st.text(alphabet="abcSs0123456789 _-eason", min_size=1, max_size=8)


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.lists(_seg, min_size=0, max_size=2),
                          st.sampled_from(["a.mkv", "b.mp4", "c.txt", "d.MOV", "e.webm"])),
                min_size=1, max_size=8),
       st.booleans())
def test_property_output_is_subset_and_media_only(tmp_path_factory, entries, movie):
    root = tmp_path_factory.mktemp("p")
    rels = set()
    for dirs, fname in entries:
        rel = os.path.join(*dirs, fname) if dirs else fname
        rels.add(rel)
    try:
        make_tree(root, sorted(rels))
    except (FileExistsError, NotADirectoryError, IsADirectoryError):
        return
    files = find_media_files(str(root), MOVIE if movie else TV)
    for f in files:
        assert os.path.isfile(f)
        assert node_extname(os.path.basename(f)) in (".mp4", ".mkv", ".mov", ".webm")
    assert len(files) == len(set(files))
    if movie:
        # MOVIE keeps every directory: all media files are selected.
        want = sum(1 for r in rels if os.path.isfile(os.path.join(root, r))
                   and node_extname(os.path.basename(r)) in (".mp4", ".mkv", ".mov", ".webm"))
        assert len(files) == want
    # top-level media files are always kept
    top = [r for r in rels if os.sep not in r and r.endswith((".mkv", ".mp4", ".webm"))
           and os.path.isfile(os.path.join(root, r))]
    for t in top:
        assert os.path.join(str(root), t) in files


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.lists(_seg, min_size=0, max_size=2),
                          st.sampled_from(["a.mkv", "b.mp4", "c.txt", "S1.mkv", "e.webm"])),
                min_size=1, max_size=8),
       st.booleans())
def test_virtual_walk_matches_disk_walk(tmp_path_factory, entries, movie):
    """find_virtual (torrent file list before download) == find (tree on disk)."""
    root = tmp_path_factory.mktemp("v")
    rels = sorted({os.path.join(*d, f) if d else f for d, f in entries})
    try:
        make_tree(root, rels)
    except (FileExistsError, NotADirectoryError, IsADirectoryError):
        return
    rels = [r for r in rels if os.path.isfile(os.path.join(root, r))]
    sel = MediaSelector()
    mt = MOVIE if movie else TV
    assert sel.find_virtual(str(root), rels, mt) == sel.find(str(root), mt)


def test_virtual_walk_reference_fixture(tmp_path):
    rels = ["Season 1/KonoSuba S1E1.mkv", "Extras/KonoSuba OVA.mkv",
            "Commentary/KonoSuba Season 1 Commentary.mkv", "S1/KonoSuba S1E1.mkv"]
    got = MediaSelector().find_virtual("/job", rels, TV)
    assert got == ["/job/S1/KonoSuba S1E1.mkv", "/job/Season 1/KonoSuba S1E1.mkv"]


def test_use_real_logger_switch(monkeypatch):
    monkeypatch.delenv("USE_REAL_LOGGER", raising=False)
    assert isinstance(make_test_logger(), NullLogger)
    monkeypatch.setenv("USE_REAL_LOGGER", "1")
    assert not isinstance(make_test_logger(), NullLogger)


def test_process_stage_many_file_torrent_is_linear(run, tmp_path):
    """A 10k-file torrent whose files were all eagerly staged: the process stage filters the
    streamed entries against the selection in linear time (it rebuilt set(files) once per
    entry - 10^8 inserts - in round 2)."""
    import time

    from downloader_amd.stages.base import Job
    from downloader_amd.stages.process import ProcessStage
    from downloader_amd.utils.config import load_config
    root = tmp_path / "job" / "Movie"
    root.mkdir(parents=True)
    n = 10_000
    for i in range(n):
        (root / f"f{i:05d}.mkv").touch()
    files = [str(root / f"f{i:05d}.mkv") for i in range(n)]
    streamed = [{"file": f, "key": f"k{i}", "size": 0} for i, f in enumerate(files)]
    msg = api.make_download("big", "torrent", "magnet:?xt=urn:btih:" + "0" * 40, "MOVIE")
    job = Job(msg=msg, media=msg.media, last_stage={"path": str(tmp_path / "job"),
                                                  "streamed": streamed})
    st = ProcessStage(load_config(env={}), None)
    t0 = time.perf_counter()
    out = run(st.run(job))
    assert time.perf_counter() - t0 < 5.0
    assert len(out["files"]) == n and len(out["streamed"]) == n
