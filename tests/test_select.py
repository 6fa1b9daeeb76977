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


# ---- predict_media: the torrent path's upload-before-walk prediction must be
# exactly what the walk returns once the files exist (service streams uploads
# per completed file and trusts it)

_NAMES = ["a.mkv", "b.mp4", "c.nfo", "d.webm", "x.MKV", "e.mov", ".mkv"]
_DIRS = ["season 1", "Show.S01", "Extras", "s2", "Season 3", "sample", "series"]


def _layouts():
    import random
    rng = random.Random(1234)
    for _ in range(300):
        n = rng.randint(1, 6)
        files = set()
        single_tld = rng.random() < 0.6
        tld = rng.choice(_DIRS)
        for _k in range(n):
            depth = rng.randint(0, 3)
            comps = [rng.choice(_DIRS) for _d in range(depth)]
            if single_tld:
                comps = [tld] + comps
            files.add("/".join(comps + [rng.choice(_NAMES)]))
        yield sorted(files)


def test_predict_media_matches_dir_media(tmp_path):
    from tritondl.select import predict_media
    for k, layout in enumerate(_layouts()):
        root = tmp_path / f"case{k}"
        root.mkdir()
        paths = [os.path.join(str(root), rel) for rel in layout]
        pred = predict_media(str(root), paths)        # before any file exists
        for p in paths:
            if any(q.startswith(p + "/") for q in paths):
                break                                 # a name used as both file and dir: not a layout
        else:
            for rel in layout:
                _touch(str(root), rel)
            _touch(str(root), ".torrent.db")          # top-level plain files never matter
            assert pred == set(dir_media(str(root))), layout


def test_predict_media_refuses_foreign_directories(tmp_path):
    from tritondl.select import predict_media
    os.makedirs(tmp_path / "leftover")
    assert predict_media(str(tmp_path), [str(tmp_path / "Show" / "season 1" / "e1.mkv")]) is None
    # a directory the torrent itself creates is fine (resume of a redelivered job)
    os.makedirs(tmp_path / "Show")
    os.rmdir(tmp_path / "leftover")
    assert predict_media(str(tmp_path), [str(tmp_path / "Show" / "season 1" / "e1.mkv")]) == \
        {str(tmp_path / "Show" / "season 1" / "e1.mkv")}


# ------------------------------------------------------- property: the rules vs a model

def _model(tree: dict) -> list[str]:
    """SURVEY.md Appendix A.1, written independently of ``select.py``: an
    in-memory tree ({name: subtree or None}) -> the relative paths
    ``process.Dir`` returns, in its order."""
    import re
    top_dirs = [n for n, v in tree.items() if isinstance(v, dict)]
    allowed = ["season"] + ([top_dirs[0]] if len(top_dirs) == 1 else [])
    out: list[str] = []

    def walk(node: dict, prefix: list[str]) -> None:
        for name in sorted(node, key=lambda n: n.encode()):           # filepath.Walk: lexical
            v = node[name]
            if isinstance(v, dict):
                if any(a in name for a in allowed) or re.search(r"s\d+", name):
                    walk(v, prefix + [name])
            else:
                dot = name.rfind(".")                                  # filepath.Ext
                if dot >= 0 and name[dot:] in (".mp4", ".mkv", ".mov", ".webm"):
                    out.append("/".join(prefix + [name]))
    walk(tree, [])
    return out


def test_dir_media_matches_the_rules_on_random_trees():
    """Random trees (names built to hit the rules' edges: "season" as a
    substring, capital S, s<digits> anywhere, the sole top-level directory,
    dotfiles, upper-case and compound extensions) give exactly the model's
    list, in its order."""
    import tempfile

    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    from tritondl.select import dir_media

    stems = st.sampled_from(["season 1", "Season 2", "my season", "s01", "S01", "xs12y", "extras", "show",
                             "a", "b", "c d", "Ab", "s", "sx", ""])
    exts = st.sampled_from([".mkv", ".mp4", ".mov", ".webm", ".MKV", ".srt", ".mkv.part", ".tar.mkv", ""])
    file_names = st.tuples(stems, exts).map(lambda t: t[0] + t[1]).filter(lambda n: n not in ("", ".", ".."))
    dir_names = stems.filter(lambda n: n not in ("", ".", ".."))
    trees = st.recursive(
        st.dictionaries(file_names, st.none(), max_size=4),
        lambda kids: st.dictionaries(dir_names | file_names, kids | st.none(), max_size=4),
        max_leaves=14).filter(lambda t: isinstance(t, dict))

    def make(root: str, node: dict) -> None:
        for name, v in node.items():
            p = os.path.join(root, name)
            if isinstance(v, dict):
                os.mkdir(p)
                make(p, v)
            else:
                with open(p, "wb"):
                    pass

    @settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
    @given(trees)
    def check(tree):
        with tempfile.TemporaryDirectory() as root:
            make(root, tree)
            got = [os.path.relpath(p, root) for p in dir_media(root)]
            assert got == _model(tree)

    check()


def test_predict_media_matches_dir_media_on_random_layouts():
    """For any torrent layout (files only; directories exist because files do),
    the prediction made from the path strings before a byte is written equals
    the real walk once every file exists."""
    import tempfile

    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    from tritondl.select import dir_media, predict_media

    stems = st.sampled_from(["season 1", "Season 2", "s01", "S01", "xs12y", "extras", "show", "a", "b c"])
    exts = st.sampled_from([".mkv", ".mp4", ".mov", ".webm", ".MKV", ".srt", ".nfo", ""])
    file_names = st.tuples(stems, exts).map(lambda t: t[0] + t[1])
    trees = st.recursive(st.dictionaries(file_names, st.none(), max_size=4),
                         lambda kids: st.dictionaries(stems | file_names, kids | st.none(), max_size=4),
                         max_leaves=14)

    def leaves(node: dict, prefix: tuple = ()) -> list[str]:
        out = []
        for name, v in node.items():
            if isinstance(v, dict):
                out += leaves(v, prefix + (name,))
            else:
                out.append("/".join(prefix + (name,)))
        return out

    @settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
    @given(trees)
    def check(tree):
        with tempfile.TemporaryDirectory() as root:
            rels = leaves(tree)
            paths = [os.path.join(root, r) for r in rels]
            pred = predict_media(root, paths)
            for r in rels:
                os.makedirs(os.path.dirname(os.path.join(root, r)), exist_ok=True)
                with open(os.path.join(root, r), "wb"):
                    pass
            assert pred == set(dir_media(root)), rels

    check()
