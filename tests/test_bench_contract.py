"""bench.py contract: one JSON line from rank 0 with the required fields,
single process and under torch.distributed.run with 2 ranks (gloo on CPU),
value = whole-job aggregate."""

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _env():
    env = dict(os.environ)
    env.update({"MASTER_ADDR": "127.0.0.1", "TRITONDL_GPU_VERIFY": "off", "PYTHONPATH": ROOT})
    return env


def test_bench_single_process_json():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--file-mb", "1",
                        "--no-gpu-probe"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert REQUIRED <= d.keys() and d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["model"].startswith("Single HTTP download job") and d["config"]["parallelism"] == "dp1"
    assert abs(d["value"] - 4 / (d["ms_per_step"] * 4 / 1000)) / d["value"] < 0.01
    # the placement is part of the reported config (default: pinned to an L3 domain)
    assert d["config"]["cpus"].endswith(")") and "pinned" in d["config"]["cpus"]
    assert d["config"]["fake_cpus"]
    # diagnostics that explain a slow lease: host page-cache counters, the work dir's
    # filesystem and spare use, and the same for the reference's cleanup-off mode
    vm = d["diag"]["vm"]
    assert "nr_dirtied_per_job" in vm and len(vm["Dirty_kB"]) == 2
    assert d["diag"]["work_fs"]["fs"] and d["diag"]["work_fs"]["spares_taken"] >= 1
    rm = d["reference_mode"]
    assert rm["cleanup"] is False and rm["fetched_ms_p50"] > 0 and "nr_dirtied_per_job" in rm["vm"]


def test_bench_two_ranks_torchrun_gloo():
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--file-mb", "1", "--no-gpu-probe"],
                       cwd=ROOT, capture_output=True, text=True, timeout=400, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2
    # whole-job aggregate: 2 ranks x 3 steps over the slowest rank's time
    assert abs(d["value"] - 2 * 3 / (d["ms_per_step"] * 3 / 1000)) / d["value"] < 0.01
    # one shared broker, competing consumers: both workers took jobs
    assert d["config"]["topology"].startswith("one shared broker")
    assert len(d["jobs_per_rank"]) == 2 and all(n > 0 for n in d["jobs_per_rank"]), d["jobs_per_rank"]
    assert sum(d["jobs_per_rank"]) == 2 * 3
    assert d["config"]["collectives"].startswith("gloo max-reduce")
    assert len(d["diag"]["placement_per_rank"]) == 2


def test_bench_dist_always_one_rank():
    """--dist-always runs the multi-rank collective path (process group,
    gloo control group, closing max-reduce) with a single rank — what a
    one-GPU box can exercise of the RCCL path."""
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--dist-always",
                        "--steps", "3", "--warmup", "1", "--file-mb", "1", "--no-gpu-probe"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    assert d["n_gpus"] == 1 and d["config"]["collectives"].startswith("gloo max-reduce")


def test_bench_tls_json():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--file-mb", "1",
                        "--no-gpu-probe", "--tls"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_lines(r.stdout)[0]
    assert d["config"]["transport"].startswith("https") and d["config"]["s3_payload"] == "unsigned"
    assert d["value"] > 0


def test_bench_tls_over_an_http2_origin_json():
    """--tls --h2-origin: every job's download is an HTTP/2 stream (the worker
    offers h2 by default) and its upload is content-checked like any other."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--file-mb", "1",
                        "--no-gpu-probe", "--tls", "--h2-origin", "--no-reference-mode"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_lines(r.stdout)[0]
    assert "HTTP/2" in d["config"]["transport"] and d["config"]["http2"] is True
    assert d["diag"]["h2_streams"] >= 5 and d["diag"]["s3_content_checked"]
