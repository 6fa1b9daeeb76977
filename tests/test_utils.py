import io
import json

from tritondl.utils.backoff import ExponentialBackoff
from tritondl.utils.config import Config
from tritondl.utils.gocompat import go_base, go_clean, go_ext, go_join
from tritondl.utils.log import Logger


def test_go_path_helpers():
    assert go_ext("a/b.tar.gz") == ".gz"
    assert go_ext("a.b/c") == ""
    assert go_ext(".mkv") == ".mkv"
    assert go_clean("/a/../b/./c//") == "/b/c"
    assert go_clean("../x/..") == ".."
    assert go_clean("/..") == "/"
    assert go_join("a", "", "b/") == "a/b"
    assert go_join("x", "original/", "Zm9v") == "x/original/Zm9v"
    assert go_base("/a/b/") == "b"


def test_config_defaults_match_reference(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    c = Config.from_env({})
    assert c.rabbitmq_endpoint == "127.0.0.1:5672" and c.rabbitmq_endpoint_defaulted
    assert c.consume_topic == "v1.download" and c.publish_topic == "v1.convert"
    assert c.bucket == "triton-staging" and c.prefetch == 1 and c.num_shard_queues == 2
    assert c.download_dir == str(tmp_path / "downloading")
    assert c.metadata_timeout_s == 600


def test_config_env_and_flags():
    env = {"RABBITMQ_ENDPOINT": "h:1", "RABBITMQ_USERNAME": "u@x", "RABBITMQ_PASSWORD": "p/w:",
           "S3_ENDPOINT": "https://s3:9000", "TRITONDL_CONCURRENCY": "4", "DOWNLOAD": "x"}
    c = Config.from_env(env, argv=["-cpuprofile", "p.prof", "--prefetch", "8"])
    assert c.rabbitmq_url() == "amqp://u%40x:p%2Fw%3A@h:1"
    assert c.cpuprofile == "p.prof" and c.prefetch == 8 and c.concurrency == 4


def test_logger_text_and_json():
    s = io.StringIO()
    lg = Logger(s)
    lg.with_fields(event="decode-message", n=3).info("hello %s", "world")
    line = s.getvalue().strip()
    assert 'level=info msg="hello world"' in line and "event=decode-message" in line and "n=3" in line
    s2 = io.StringIO()
    lg2 = Logger(s2)
    lg2.configure("debug", "json")
    lg2.with_field("url", "http://x").debug("download status")
    rec = json.loads(s2.getvalue())
    assert rec["level"] == "debug" and rec["url"] == "http://x" and "file" in rec and "func" in rec


def test_logger_level_filter():
    s = io.StringIO()
    lg = Logger(s)
    lg.debug("nope")
    assert s.getvalue() == ""


def test_backoff_grows_and_caps():
    b = ExponentialBackoff(initial=1, multiplier=2, randomization=0, max_interval=5, max_elapsed=None)
    assert [b.next_delay() for _ in range(5)] == [1, 2, 4, 5, 5]
    b2 = ExponentialBackoff(max_elapsed=0.0)
    import time
    time.sleep(0.01)
    assert b2.next_delay() is None


def test_durafmt_matches_hako_durafmt_format():
    from tritondl.utils.gocompat import durafmt
    assert durafmt(10) == "10 seconds"
    assert durafmt(1) == "1 second"
    assert durafmt(90.5) == "1 minute 30 seconds 500 milliseconds"
    assert durafmt(0) == "0 seconds"
    assert durafmt(3600 * 25) == "1 day 1 hour"
    assert durafmt(0.000002) == "2 microseconds"


def test_config_data_plane_knobs():
    from tritondl.utils.config import Config
    c = Config.from_env({})
    assert (c.http_probe_bytes, c.http_segments, c.s3_sign_threads) == (0, 4, 4)
    c = Config.from_env({"TRITONDL_HTTP_PROBE_BYTES": "4194304", "TRITONDL_HTTP_SEGMENTS": "8",
                         "TRITONDL_HTTP_SEGMENT_THRESHOLD": "1048576", "TRITONDL_S3_SIGN_THREADS": "2"})
    assert (c.http_probe_bytes, c.http_segments, c.http_segment_threshold, c.s3_sign_threads) == \
        (4 << 20, 8, 1 << 20, 2)
