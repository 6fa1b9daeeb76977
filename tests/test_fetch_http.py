"""Dispatcher routing (reference downloader.go:138-176 semantics) and the
HTTP downloader against the fake origin: naming, resume, segmentation,
retries, error surfacing."""

import asyncio
import os

import pytest

from tritondl_testkit.fakes.origin import Origin
from tritondl.fetch.http import HTTPDownloader, HTTPDownloadError, filename_from_disposition
from tritondl.fetch.registry import ClientRegister, Dispatcher, ProgressTracker, UnsupportedError


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


class FakeImpl:
    def __init__(self, name, protocols=(), exts=()):
        self.reg = ClientRegister(name, list(protocols), list(exts))
        self.calls = []

    def register(self):
        return self.reg

    async def download(self, base_dir, progress, url):
        self.calls.append((base_dir, url))
        progress(url, 50)
        progress(url, 100)


def test_dispatch_rules(tmp_path):
    torrent = FakeImpl("torrent", ["magnet"], [".torrent"])
    http = FakeImpl("http", ["http", "https"])
    d = Dispatcher(str(tmp_path), [torrent, http])
    assert d.select("magnet:?xt=urn:btih:abc") is torrent
    assert d.select("http://h/x/file.torrent") is torrent        # ext wins for http(s)
    assert d.select("https://h/movie.mkv") is http
    assert d.select("https://h/movie.torrent?x=1") is torrent
    with pytest.raises(UnsupportedError) as ei:
        d.select("ftp://h/a.zip")
    assert str(ei.value) == "unsupported fileext '.zip' or protocol 'ftp'"
    with pytest.raises(UnsupportedError):
        d.select("ftp://h/a.torrent")                              # ext only applies to http(s)
    with pytest.raises(ValueError, match="invalid baseDir"):
        Dispatcher("relative/dir", [http])
    out = run(d.download("job1", "http://h/f.mkv"))
    assert out == str(tmp_path / "job1") and os.path.isdir(out)
    assert http.calls == [(out, "http://h/f.mkv")]
    with pytest.raises(ValueError):
        d.job_dir("../escape")


def test_progress_tracker_drops_at_100():
    t = ProgressTracker(interval=0)
    from tritondl.fetch.registry import ProgressUpdate
    t.update(ProgressUpdate("u", 10))
    assert t.progress == {"u": 10}
    t.update(ProgressUpdate("u", 100))
    assert t.progress == {}


def test_content_disposition():
    assert filename_from_disposition('attachment; filename="a b.mkv"') == "a b.mkv"
    assert filename_from_disposition("attachment; filename*=UTF-8''%C3%A9t%C3%A9.mp4") == "été.mp4"
    assert filename_from_disposition('attachment; filename="../../etc/passwd"') == "passwd"


class Sink:
    def __init__(self):
        self.events = []

    def __call__(self, url, p):
        self.events.append(p)


def _dl(**kw):
    kw.setdefault("progress_interval", 0.01)
    return HTTPDownloader(**kw)


def test_http_download_basic_and_skip_existing(tmp_path):
    async def main():
        o = await Origin().start()
        data = os.urandom(3_000_000)
        url = o.add("/media/Movie%20One.mkv", data)
        h = _dl()
        s = Sink()
        await h.download(str(tmp_path), s, url)
        assert (tmp_path / "Movie One.mkv").read_bytes() == data
        assert s.events[-1] == 100 and not (tmp_path / "Movie One.mkv.part").exists()
        n = len(o.requests)
        await h.download(str(tmp_path), s, url)       # already complete: only the probe (closed unread)
        assert [r[0] for r in o.requests[n:]] == ["GET"]
        h2 = _dl(probe="head")                         # grab's order: HEAD first
        n = len(o.requests)
        await h2.download(str(tmp_path), s, url)
        assert [r[0] for r in o.requests[n:]] == ["HEAD"]
        await h2.close()
        await h.close()
        await o.stop()
    run(main())


def test_http_disposition_name_and_no_head(tmp_path):
    async def main():
        o = await Origin().start()
        o.head = False
        url = o.add("/dl", b"abc" * 1000, disposition='attachment; filename="show.s01e01.mkv"')
        h = _dl()
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "show.s01e01.mkv").read_bytes() == b"abc" * 1000
        await h.close()
        await o.stop()
    run(main())


def test_http_resume_after_cut(tmp_path):
    async def main():
        o = await Origin().start()
        data = os.urandom(5_000_000)
        url = o.add("/f.mp4", data)
        o.cut_after, o.cut_times = 1_500_000, 1
        h = _dl(max_retries=0, write_block=256 * 1024)
        with pytest.raises(HTTPDownloadError):
            await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "f.mp4.part").exists() and (tmp_path / "f.mp4.part.meta").exists()
        h2 = _dl()
        await h2.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "f.mp4").read_bytes() == data
        ranges = [r[2] for r in o.requests if r[0] == "GET"]
        assert ranges[-1].startswith("bytes=") and ranges[-1] != "bytes=0-"
        await h.close()
        await h2.close()
        await o.stop()
    run(main())


def _gap(m):
    m["segments"] = [[a + 1, b, 0] for a, b, _d in m["segments"]]
    return m


@pytest.mark.parametrize("tamper", [
    _gap, lambda m: [m], lambda m: {**m, "segments": "x"},
    lambda m: {**m, "segments": [[0, m["size"], -1]]}, lambda m: {**m, "segments": [[0, 1.5, 0]]}])
def test_http_resume_ignores_a_plan_that_does_not_tile_the_file(tmp_path, tamper):
    """A ``.part.meta`` whose segments do not tile [0, size) with sane done
    counts (hand-edited, or written by another version) restarts the
    download instead of leaving holes in the file or crashing."""
    import json

    async def main():
        o = await Origin().start()
        data = os.urandom(5_000_000)
        url = o.add("/f.mp4", data)
        o.cut_after, o.cut_times = 1_500_000, 1
        h = _dl(max_retries=0, write_block=256 * 1024)
        with pytest.raises(HTTPDownloadError):
            await h.download(str(tmp_path), Sink(), url)
        mp = tmp_path / "f.mp4.part.meta"
        mp.write_text(json.dumps(tamper(json.loads(mp.read_text()))))
        h2 = _dl()
        await h2.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "f.mp4").read_bytes() == data
        await h.close()
        await h2.close()
        await o.stop()
    run(main())


def test_http_in_process_retry_and_segments(tmp_path):
    async def main():
        o = await Origin().start()
        data = os.urandom(9_000_000)
        url = o.add("/big.webm", data)
        o.cut_after, o.cut_times = 700_000, 2
        h = _dl(segments=4, segment_threshold=1_000_000, write_block=512 * 1024)
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "big.webm").read_bytes() == data
        gets = [r for r in o.requests if r[0] == "GET"]
        assert len({r[2] for r in gets}) >= 4
        await h.close()
        await o.stop()
    run(main())


def test_http_errors_surface(tmp_path):
    async def main():
        o = await Origin().start()
        h = _dl(max_retries=1)
        with pytest.raises(Exception):
            await h.download(str(tmp_path), Sink(), o.url("/missing.mkv"))
        url = o.add("/x.mkv", b"z" * 10)
        o.fail = 1  # the probe gets a 500 -> retried
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "x.mkv").read_bytes() == b"z" * 10
        hh = _dl(max_retries=1, probe="head")
        o.fail = 1  # HEAD gets 500 -> falls back to ranged GET probe
        os.remove(tmp_path / "x.mkv")
        await hh.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "x.mkv").read_bytes() == b"z" * 10
        await hh.close()
        await h.close()
        await o.stop()
    run(main())


def test_get_probe_empty_file_and_rangeless_origin(tmp_path):
    async def main():
        o = await Origin().start()
        h = _dl()
        url = o.add("/empty.mkv", b"")
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "empty.mkv").read_bytes() == b""
        o.ranges = False                           # origin ignores Range: 200 + full body
        data = os.urandom(200_000)
        url2 = o.add("/full.mkv", data)
        n = len(o.requests)
        await h.download(str(tmp_path), Sink(), url2)
        assert (tmp_path / "full.mkv").read_bytes() == data
        assert [r[0] for r in o.requests[n:]] == ["GET"]      # the probe WAS the download
        await h.close()
        await o.stop()
    run(main())


def test_get_probe_saves_a_round_trip(tmp_path):
    """With a distant origin the default probe (ranged GET kept open as the
    data stream) finishes a small download a whole request latency sooner
    than grab's HEAD-then-GET."""
    async def main():
        import time as _t
        o = await Origin().start()
        o.latency = 0.15
        url = o.add("/clip.mkv", os.urandom(10_000))
        times = {}
        for mode in ("head", "get"):
            h = _dl(probe=mode)
            d = tmp_path / mode
            os.makedirs(d)
            t0 = _t.perf_counter()
            await h.download(str(d), Sink(), url)
            times[mode] = _t.perf_counter() - t0
            await h.close()
        assert times["head"] - times["get"] > 0.1, times
        await o.stop()
    run(main())


def test_bounded_probe_segments_mid_size_files(tmp_path):
    """``probe_bytes``: the GET probe asks for ``bytes=0-(N-1)``; a bigger file's
    rest is requested at once as up to ``segments`` Range streams, a file that
    fits the probe stays one request, and a Range-ignoring origin still works."""
    async def main():
        o = await Origin().start()
        pb = 512 * 1024
        h = _dl(segments=4, probe_bytes=pb, write_block=256 * 1024)
        data = os.urandom(3_000_000)
        url = o.add("/mid.mkv", data)
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "mid.mkv").read_bytes() == data
        rngs = [r[2] for r in o.requests if r[0] == "GET"]
        assert rngs[0] == f"bytes=0-{pb - 1}"
        assert len(rngs) == 4 and all(r.startswith("bytes=") for r in rngs)   # probe + segments-1
        small = os.urandom(100_000)
        n = len(o.requests)
        url2 = o.add("/small.mkv", small)
        await h.download(str(tmp_path), Sink(), url2)
        assert (tmp_path / "small.mkv").read_bytes() == small
        assert len(o.requests[n:]) == 1
        o.ranges = False
        url3 = o.add("/plain.mkv", data)
        n = len(o.requests)
        await h.download(str(tmp_path), Sink(), url3)
        assert (tmp_path / "plain.mkv").read_bytes() == data
        assert len(o.requests[n:]) == 1
        await h.close()
        await o.stop()
    run(main())


def test_bounded_probe_plan_covers_file():
    from tritondl.fetch.http import _Probe
    h = HTTPDownloader(segments=4, probe_bytes=1000)
    for size, first in ((999, 999), (1000, 1000), (1001, 1000), (2500, 1000), (10_007, 1000)):
        p = _Probe(size=size, ranges=True, etag="", last_modified="", filename="f", status=206, first_end=first)
        segs = h._plan(p)
        assert segs[0][:2] == [0, first]
        assert all(a[1] == b[0] for a, b in zip(segs, segs[1:]))
        assert segs[-1][1] == size and len(segs) <= 5


def test_failed_segment_stops_and_awaits_sibling_pumps(tmp_path):
    """One Range stream dies for good while its siblings sit in their native
    pumps (the origin sends 1 MiB bursts with pauses).  By the time the
    download raises, every sibling pump must have returned — the .part fd and
    the sockets are closed only then, so no pump can write through a recycled
    fd number (another job's file, the AMQP socket).  A concurrent download of
    another file is unaffected."""
    from tritondl.utils import rawhttp

    async def main():
        o = await Origin().start()
        data = os.urandom(12_000_000)
        other = os.urandom(4_000_000)
        url = o.add("/seg/bad.mkv", data)
        url2 = o.add("/seg/good.mkv", other)
        o.rate = 2_000_000                       # siblings idle between 1 MiB bursts when one is cut
        # segment 2 dies after its first burst, while segments 0, 1, 3 are mid-body
        o.cut_after, o.cut_times, o.cut_match = 1_500_000, 1, "bytes=6000000-"
        h = _dl(segments=4, segment_threshold=1 << 20, max_retries=0)
        d1, d2 = tmp_path / "a", tmp_path / "b"
        d1.mkdir()
        d2.mkdir()
        with pytest.raises(HTTPDownloadError):
            await h.download(str(d1), Sink(), url)
        assert rawhttp.active_pumps() == 0, "sibling pumps still running after the download failed"
        part = d1 / "bad.mkv.part"
        size0, mtime0 = part.stat().st_size, part.stat().st_mtime_ns
        await asyncio.sleep(0.6)                 # the origin keeps sending: nothing may land anywhere
        assert part.stat().st_mtime_ns == mtime0 and part.stat().st_size == size0
        # concurrency: one download fails while another runs to completion
        o.cut_after, o.cut_times, o.cut_match = 1_500_000, 0, "bytes=6000000-"
        good = asyncio.ensure_future(_dl(segments=4, segment_threshold=1 << 20).download(str(d2), Sink(), url2))
        await asyncio.sleep(0.05)
        o.cut_times = 1
        bad = asyncio.ensure_future(h.download(str(d1), Sink(), url))
        res = await asyncio.gather(good, bad, return_exceptions=True)
        assert (d2 / "good.mkv").read_bytes() == other
        assert res[0] is None
        await h.close()
        await o.stop()
    run(main(), timeout=90)


def test_striped_streams_pull_stripes_in_order(tmp_path):
    """``stripe_bytes``: ``segments`` stream workers take fixed-size stripes in
    file order over their keep-alive connections — the file is complete and
    correct, every stripe is one Range request, the stripes are requested in
    ascending order, and an interrupted striped download resumes."""
    async def main():
        o = await Origin().start()
        pb, st = 256 * 1024, 300_000
        h = _dl(segments=3, probe_bytes=pb, stripe_bytes=st, write_block=128 * 1024)
        data = os.urandom(2_500_000)
        url = o.add("/striped.mkv", data)
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "striped.mkv").read_bytes() == data
        rngs = [r[2] for r in o.requests if r[0] == "GET"]
        assert rngs[0] == f"bytes=0-{pb - 1}"
        starts = [int(r.split("=")[1].split("-")[0]) for r in rngs[1:]]
        want = list(range(pb, len(data), st))
        assert sorted(starts) == want
        # taken in file order: at most `segments` stripes are ever in flight out of turn
        assert all(want.index(x) <= k + 2 for k, x in enumerate(starts)), starts
        # HEAD-probe plan (open-ended probe) stripes files above the threshold too
        plan = HTTPDownloader(segments=4, segment_threshold=1000, stripe_bytes=400)._plan(
            __import__("tritondl.fetch.http", fromlist=["_Probe"])._Probe(
                size=1900, ranges=True, etag="", last_modified="", filename="f", status=200))
        assert plan == [[0, 400, 0], [400, 800, 0], [800, 1200, 0], [1200, 1600, 0], [1600, 1900, 0]]
        # a cut mid-stripe fails the job; the next attempt resumes from the meta
        url2 = o.add("/cut.mkv", data)
        o.cut_after, o.cut_times, o.cut_match = 100_000, 1, f"bytes={pb + st}-"
        h0 = _dl(segments=3, probe_bytes=pb, stripe_bytes=st, max_retries=0)
        with pytest.raises(HTTPDownloadError):
            await h0.download(str(tmp_path), Sink(), url2)
        n = len(o.requests)
        await h.download(str(tmp_path), Sink(), url2)
        assert (tmp_path / "cut.mkv").read_bytes() == data

        def span(r: str) -> int:
            a, b = r.split("=")[1].split("-")
            return (int(b) + 1 if b else len(data)) - int(a)
        # resumed, not refetched from zero: after its probe, the second attempt asks for
        # less than the part beyond the probe (which stripes had finished when the cut
        # came is a race; the cut stripe's first 100,000 bytes are always kept)
        again = [r[2] for r in o.requests[n:] if r[0] == "GET"][1:]
        assert sum(span(r) for r in again) < len(data) - pb, again
        await h0.close()
        await h.close()
        await o.stop()
    run(main())


def test_redirects_followed_natively(tmp_path):
    """301 -> 307 chains (absolute and relative Location) are followed on the
    native path; the file is named after the FINAL URL (grab / Go http.Client
    behaviour); later Range requests go straight to the final URL; a loop
    stops after max_redirects."""
    async def main():
        from tritondl.fetch import http as H
        o = await Origin().start()
        data = os.urandom(1_500_000)
        o.add("/cdn/real-name.mkv", data)
        o.redirect("/b/hop2", "/cdn/real-name.mkv", 307)                 # relative
        o.redirect("/a/watch", o.url("/b/hop2"), 301)                   # absolute
        start = o.url("/a/watch") + "?id=7"
        h = _dl(segments=3, probe_bytes=256 * 1024)
        fell_back = []
        orig_raw = h._raw_get

        async def spy(url, headers):
            r = await orig_raw(url, headers)
            fell_back.append(r is None)
            return r
        h._raw_get = spy
        await h.download(str(tmp_path), Sink(), start)
        assert (tmp_path / "real-name.mkv").read_bytes() == data
        assert fell_back and not any(fell_back)                        # never left the native path
        paths = [r[1] for r in o.requests if r[0] == "GET"]
        assert paths[:3] == ["/a/watch", "/b/hop2", "/cdn/real-name.mkv"]
        assert all(p == "/cdn/real-name.mkv" for p in paths[3:]) and len(paths) > 3   # ranges skip the hops
        o.redirect("/loop", "/loop")
        with pytest.raises(H.HTTPDownloadError):
            await _dl(max_retries=0).download(str(tmp_path), Sink(), o.url("/loop"))
        o.redirect("/bad", "http://[::1")                                  # unparsable Location
        with pytest.raises(H.HTTPDownloadError, match="bad redirect Location"):
            await _dl(max_retries=0).download(str(tmp_path), Sink(), o.url("/bad"))
        await h.close()
        await o.stop()
    run(main())


def test_disk_space_preflight_fails_fast(tmp_path, monkeypatch):
    """A download that cannot fit fails before writing anything (the reference
    let grab fill the disk); a resumed download only needs what is missing."""
    async def main():
        from tritondl.utils import disk
        o = await Origin().start()
        data = os.urandom(400_000)
        url = o.add("/big.mkv", data)
        monkeypatch.setattr(disk, "free_bytes", lambda p: 300_000)
        with pytest.raises(HTTPDownloadError, match="not enough disk space"):
            await _dl().download(str(tmp_path), Sink(), url)
        assert not (tmp_path / "big.mkv.part").exists()
        monkeypatch.setattr(disk, "free_bytes", lambda p: 10**12)
        h = _dl(disk_reserve=10**12 - 100_000)          # the reserve counts too
        with pytest.raises(HTTPDownloadError, match="reserve"):
            await h.download(str(tmp_path), Sink(), url)
        await _dl().download(str(tmp_path), Sink(), url)
        assert (tmp_path / "big.mkv").read_bytes() == data
        await o.stop()
    run(main())


@pytest.mark.parametrize("native", [True, False])
def test_chunked_origin_fetched_once(tmp_path, native):
    """A chunked response (no length, no ranges; chunk extensions and a
    trailer) is decoded by the native receive pump — one GET, no second
    request through aiohttp — and the keep-alive connection is reused."""
    from tritondl.utils import rawhttp

    async def main():
        o = await Origin().start()
        o.chunked = True
        data = os.urandom(2_345_678)
        url = o.add("/live/feed.mkv", data)
        h = _dl(native=native, segments=4)
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "feed.mkv").read_bytes() == data
        assert [r[0] for r in o.requests] == ["GET"]                       # exactly one GET
        if native:
            assert sum(len(v) for v in h._raw.idle.values()) == 1          # read to its end: pooled
        os.remove(tmp_path / "feed.mkv")
        await h.download(str(tmp_path), Sink(), url)                      # again, on the pooled connection
        assert (tmp_path / "feed.mkv").read_bytes() == data and len(o.requests) == 2
        await h.close()
        await o.stop()
    assert rawhttp.relay_module() is not None
    run(main())


def test_chunked_decoder_rejects_bad_framing(tmp_path):
    """Malformed chunk framing fails the pump with a clear error."""
    import socket

    from tritondl.utils import rawhttp
    relay = rawhttp.relay_module()
    good = b"5;x=y\r\nhello\r\n1\r\n \r\n0\r\nT: v\r\n\r\n"
    fd = os.open(tmp_path / "out", os.O_RDWR | os.O_CREAT, 0o644)
    try:
        for body, want in ((good, ""), (b"zz\r\n", "chunk size"), (b"3\r\nabcX\r\n", "CRLF"),
                           (b"3\r\nabc\r\n", "closed inside")):
            a, b = socket.socketpair()
            a.sendall(body)
            a.close()
            got, _eof, err, reusable = relay.recv_body(b.fileno(), fd, 0, -1, b"", None, chunked=True)
            b.close()
            assert (want in err) if want else err == "", (body, err)
            if not want:
                assert got == 6 and reusable and os.pread(fd, 6, 0) == b"hello "
        a, b = socket.socketpair()                    # a cap (the segment's end) stops early, not reusable
        a.sendall(good)
        got, _eof, err, reusable = relay.recv_body(b.fileno(), fd, 0, 3, b"", None, chunked=True)
        a.close()
        b.close()
        assert (got, err, reusable) == (3, "", False)
    finally:
        os.close(fd)


def test_cancelled_fallback_download_writes_nothing_after_close(tmp_path, monkeypatch):
    """The aiohttp data path (no native relay) writes through executor threads:
    cancelling a download with several segments in flight must wait for every
    write before the file's descriptor is closed — a sentinel file opened
    right after (taking the freed descriptor number) stays untouched."""
    import time as _time

    from tritondl.fetch import http as H
    real = H._pwritev_all
    writing = []

    def slow_write(fd, bufs, pos):
        writing.append(fd)
        _time.sleep(0.3)                              # a slow disk: the write outlives the cancel
        real(fd, bufs, pos)
    monkeypatch.setattr(H, "_pwritev_all", slow_write)

    async def main():
        o = await Origin().start()
        o.rate = 8e6
        data = os.urandom(8 << 20)
        url = o.add("/big.mkv", data)
        h = _dl(native=False, segments=4, segment_threshold=1 << 20, write_block=64 << 10)
        dh = await h.start(str(tmp_path), Sink(), url)
        for _ in range(200):
            if writing:
                break
            await asyncio.sleep(0.01)
        assert writing
        dh.cancel()
        with pytest.raises(BaseException):
            await dh.wait()
        sentinels = [os.open(tmp_path / f"sentinel{k}", os.O_RDWR | os.O_CREAT, 0o644) for k in range(8)]
        await asyncio.sleep(0.8)                      # any write still in flight would land now
        for fd in sentinels:
            assert os.fstat(fd).st_size == 0
            os.close(fd)
        await h.close()
        await o.stop()
    run(main())


@pytest.mark.parametrize("native", [True, False])
def test_chunked_overrides_a_bogus_content_length(tmp_path, native):
    """RFC 9112 §6.3: with Transfer-Encoding chunked, Content-Length is
    ignored.  A server sending both (and a CL smaller than the body) must not
    truncate an open-ended download, and its connection is not reused.  (The
    aiohttp fallback refuses such a response outright: an error, never a
    silently short file.)"""
    async def main():
        o = await Origin().start()
        o.chunked = True
        o.chunked_content_length = 1000
        data = os.urandom(1_234_567)
        url = o.add("/live/both.mkv", data)
        h = _dl(native=native, segments=4)
        if not native:
            with pytest.raises(HTTPDownloadError, match="Content-Length can't be present"):
                await h.download(str(tmp_path), Sink(), url)
            await h.close()
            await o.stop()
            return
        await h.download(str(tmp_path), Sink(), url)
        assert (tmp_path / "both.mkv").read_bytes() == data
        if native:
            assert sum(len(v) for v in h._raw.idle.values()) == 0         # ambiguous framing: not pooled
        await h.close()
        await o.stop()
    run(main())


def test_retry_after_is_waited_out_inside_the_job(tmp_path):
    """429 / 503 with a short Retry-After: the download waits that long and
    retries inside the job (grab gave up on any status); a long one fails
    the job at once, for the broker-side retry path to re-run later."""
    import time as _t
    from tritondl.fetch.http import HTTPDownloadError, retry_after

    async def main():
        o = await Origin().start()
        data = os.urandom(200_000)
        url = o.add("/t.mkv", data)
        o.throttle = (2, 429, "1")
        h = HTTPDownloader(progress_interval=0.05)
        t0 = _t.monotonic()
        await h.download(str(tmp_path), Sink(), url)
        assert 1.9 <= _t.monotonic() - t0 < 6
        assert (tmp_path / "t.mkv").read_bytes() == data
        o.throttle = (1, 503, "3600")
        t0 = _t.monotonic()
        with pytest.raises(HTTPDownloadError, match="retry after 3600"):
            await HTTPDownloader(progress_interval=0.05).download(str(tmp_path / "b"), Sink(), url)
        assert _t.monotonic() - t0 < 2
        await o.stop()

    class R:
        status = 429
        headers = {"Retry-After": "Wed, 21 Oct 2015 07:28:00 GMT"}
    assert retry_after(R()) == 0.0                       # a date in the past: retry now
    R.headers = {"Retry-After": "12"}
    assert retry_after(R()) == 12.0
    R.status = 500
    assert retry_after(R()) is None
    run(main())


@pytest.mark.parametrize("native", [True, False])
def test_url_userinfo_is_sent_as_basic_auth(tmp_path, native):
    """Go's http.Client (under grab) sends a source URL's userinfo as
    ``Authorization: Basic`` on every request for that URL; the password is
    percent-decoded first, never put on the request line, and never logged."""
    import io
    from tritondl.utils.log import log

    async def main():
        o = await Origin().start()
        data = os.urandom(1_200_000)
        o.add("/private/show.mkv", data)
        o.basic_auth["/private/show.mkv"] = "alice:p@ss w0rd"
        url = o.url("/private/show.mkv").replace("http://", "http://alice:p%40ss%20w0rd@")
        h = _dl(segments=3, probe_bytes=256 * 1024, native=native)
        os.makedirs(tmp_path / "ok")
        os.makedirs(tmp_path / "no")
        await h.download(str(tmp_path / "ok"), Sink(), url)
        assert (tmp_path / "ok" / "show.mkv").read_bytes() == data
        gets = [a for (m, _p, _r), a in zip(o.requests, o.auth_seen) if m == "GET"]
        assert len(gets) >= 3 and all(a.startswith("Basic ") for a in gets)
        # no credentials: the origin's 401 fails the job
        with pytest.raises(HTTPDownloadError):
            await _dl(max_retries=0, native=native).download(str(tmp_path / "no"), Sink(),
                                                              o.url("/private/show.mkv"))
        await h.close()
        await o.stop()
    run(main())
    buf = io.StringIO()
    old = log.stream
    log.stream = buf
    try:
        log.with_field("url", "https://alice:s3cret@media.example/x.mkv").info("download status")
        log.error("dial amqp://guest:guest@rabbit:5672/ failed")
    finally:
        log.stream = old
    out = buf.getvalue()
    assert "s3cret" not in out and "guest:guest" not in out
    assert "alice:xxxxx@media.example" in out and "guest:xxxxx@rabbit" in out


def test_idle_pooled_connections_expire_and_are_capped():
    """The keep-alive pool closes a connection idle past ``idle_s`` (Go's
    IdleConnTimeout, 90 s) and keeps at most ``max_idle_total``, oldest
    closed first, so a worker that meets many origins does not hoard fds."""
    import socket
    import time as _t
    from tritondl.utils import rawhttp

    async def main():
        pool = rawhttp.Pool(idle_s=0.05, max_idle_total=2)
        pairs = [socket.socketpair() for _ in range(3)]
        conns = [rawhttp.RawConn(a) for a, _b in pairs]
        for i, c in enumerate(conns):
            pool.release(f"origin{i}", 443, c)
            _t.sleep(0.001)
        assert conns[0].sock.fileno() == -1                      # the oldest went over the cap
        assert sum(len(v) for v in pool.idle.values()) == 2
        await asyncio.sleep(0.1)
        pool.sweep(force=True)
        assert not pool.idle and all(c.sock.fileno() == -1 for c in conns)
        for _a, b in pairs:
            b.close()
    asyncio.run(main())


def test_many_origins_leave_a_bounded_number_of_sockets(tmp_path):
    """300 downloads from 300 distinct origins (127.0.x.y, one server bound
    to all of loopback): the keep-alive pool keeps at most its cap of idle
    sockets, so the worker's fds do not grow with the origins it has met."""
    from tritondl_testkit.fakes.origin import Origin

    async def main():
        o = await Origin(host="0.0.0.0").start()
        data = os.urandom(20_000)
        o.add("/m.mkv", data)
        dl = HTTPDownloader(progress_interval=1.0)
        dl._raw.max_idle_total = 40
        fds0 = len(os.listdir("/proc/self/fd"))
        for i in range(300):
            d = tmp_path / str(i)
            d.mkdir()
            await dl.download(str(d), lambda u, p: None, f"http://127.0.{i // 250}.{i % 250 + 1}:{o.port}/m.mkv")
        assert sum(len(v) for v in dl._raw.idle.values()) <= 40
        # the in-process origin holds the far end of each pooled socket: 2 fds per idle connection
        assert len(os.listdir("/proc/self/fd")) - fds0 < 2 * 40 + 20
        assert (tmp_path / "299" / "m.mkv").read_bytes() == data
        await dl.close()
        await o.stop()
    asyncio.run(main())
