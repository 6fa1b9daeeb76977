"""Golden parity tests for the media selector.

The three cases mirror the reference's only test,
``internal/process/process_test.go:25-48`` (fixtures re-created as zero-byte
files under tests/testdata/process/), followed by rule-level tests of
``process.go:41-84`` semantics.
"""

import os

import pytest

from tritondl.select import dir_media

from .conftest import TESTDATA

P = os.path.join(TESTDATA, "process")


def test_should_find_a_movie():
    assert dir_media(os.path.join(P, "movie")) == [os.path.join(P, "movie/movie.mkv")]


def test_should_find_a_movie_in_a_top_level_directory():
    assert dir_media(os.path.join(P, "movie-tld")) == [os.path.join(P, "movie-tld/movie/movie.mkv")]


def test_should_find_files_in_sub_directories():
    assert dir_media(os.path.join(P, "seasons-subdir")) == [
        os.path.join(P, "seasons-subdir/season 1/e1.mkv"),
        os.path.join(P, "seasons-subdir/season 2/e1.mkv"),
    ]


def test_missing_root_is_error(tmp_path):
    with pytest.raises(OSError):
        dir_media(str(tmp_path / "nope"))


def test_empty_returns_empty_list(tmp_path):
    assert dir_media(str(tmp_path)) == []


def _touch(root, rel):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    open(p, "wb").close()
    return p


def test_rules(tmp_path):
    r = str(tmp_path)
    keep = [
        _touch(r, "Extras1/a.mp4"),          # matches s\d+ (quirk kept)
        _touch(r, "a.webm"),
        _touch(r, "b.mov"),
        _touch(r, "my season x/s2/season 9/e.mkv"),  # nested allowed dirs
        _touch(r, "s01/e1.mkv"),
    ]
    drop = [
        _touch(r, "Season 1/e.mkv"),          # capital S pruned (not sole TLD)
        _touch(r, "c.MKV"),                   # case-sensitive extension
        _touch(r, "extras/x.mkv"),
        _touch(r, "my season x/deep/season 9/x.mkv"),  # "deep" pruned
        _touch(r, "readme.txt"),
    ]
    got = dir_media(r)
    assert sorted(got) == sorted(keep)
    assert not set(drop) & set(got)
    # lexical walk order (filepath.Walk sorts names byte-wise)
    assert got == sorted(got, key=lambda s: [os.fsencode(x) for x in s.split("/")])


def test_sole_tld_descended_case_sensitive_contains(tmp_path):
    r = str(tmp_path)
    a = _touch(r, "Show Name/Show Name S1/e.mkv")  # sub contains TLD name
    _touch(r, "Show Name/junk/e.mkv")
    assert dir_media(r) == [a]


def test_dotfile_extension_like_go(tmp_path):
    r = str(tmp_path)
    a = _touch(r, ".mkv")  # Go: filepath.Ext(".mkv") == ".mkv"
    assert dir_media(r) == [a]


def test_trailing_slash_root_is_cleaned(tmp_path):
    r = str(tmp_path)
    a = _touch(r, "x.mp4")
    assert dir_media(r + "/") == [a]
