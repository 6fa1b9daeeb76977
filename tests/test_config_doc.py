"""docs/CONFIG.md lists every environment variable the worker reads, and is
regenerated from tritondl/utils/config.py (tools/gen_config_doc.py)."""

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_doc_is_current():
    r = subprocess.run([sys.executable, "tools/gen_config_doc.py", "--check"], cwd=ROOT, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr


def test_every_setting_has_a_description():
    """A field without a comment in config.py lands in CONFIG.md with a
    blank description: every row's last cell must say something."""
    doc = open(os.path.join(ROOT, "docs", "CONFIG.md")).read()
    blank = [ln.split("|")[1].strip() for ln in doc.splitlines()
             if ln.startswith("| `TRITONDL_") and ln.rstrip().endswith("|  |")]
    assert not blank, blank


def test_every_env_name_in_the_sources_is_documented():
    doc = open(os.path.join(ROOT, "docs", "CONFIG.md")).read()
    names = set()
    for top in ("tritondl", "csrc"):
        for dirpath, _dirs, files in os.walk(os.path.join(ROOT, top)):
            for f in files:
                if f.endswith((".py", ".h", ".cpp", ".hip")):
                    with open(os.path.join(dirpath, f), errors="replace") as fh:
                        names |= set(re.findall(r"TRITONDL_[A-Z0-9_]*[A-Z0-9]", fh.read()))
    missing = sorted(n for n in names if f"`{n}`" not in doc)
    assert not missing, missing


def test_every_mapped_setting_parses():
    """Each TRITONDL_<KEY> in the maps reaches its Config field."""
    from tritondl.utils import config as C
    env = {}
    for k in C.ENV_INTS:
        env["TRITONDL_" + k] = "7"
    for k in C.ENV_FLOATS:
        env["TRITONDL_" + k] = "2.5"
    for k in C.ENV_BOOLS:
        env["TRITONDL_" + k] = "0" if getattr(C.Config(), C.ENV_BOOLS[k]) else "1"
    env["TRITONDL_S3_HASH_DEVICE"], env["TRITONDL_BT_ENCRYPTION"] = "gpu", "require"
    c = C.Config.from_env(env)
    assert all(getattr(c, f) == 7 for f in C.ENV_INTS.values())
    assert all(getattr(c, f) == 2.5 for f in C.ENV_FLOATS.values())
    assert all(getattr(c, f) != getattr(C.Config(), f) for f in C.ENV_BOOLS.values())
    assert (c.s3_hash_device, c.bt_encryption) == ("gpu", "require")


def test_every_metric_family_has_help_and_type():
    """Each metric the worker or the pool records has a HELP line, and the
    exposition carries one HELP/TYPE pair per family."""
    from tritondl.utils.metrics import HELP, Metrics
    used = set()
    for dirpath, _dirs, files in os.walk(os.path.join(ROOT, "tritondl")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                for kind, name in re.findall(r"metrics\.(inc|set|observe)\(\"([a-z_]+)\"", src):
                    used.add(name + "_total" if kind == "inc" else name)
    assert used and used <= set(HELP), sorted(used - set(HELP))
    m = Metrics()
    m.inc("jobs", status="ok")
    m.inc("jobs", status="failed", stage='say "hi"\n')
    m.set("jobs_inflight", 1)
    m.observe("stage_seconds", 0.2, stage="upload")
    text = m.render()
    for fam, kind in (("tritondl_jobs_total", "counter"), ("tritondl_jobs_inflight", "gauge"),
                      ("tritondl_stage_seconds", "histogram"), ("tritondl_uptime_seconds", "gauge")):
        assert text.count(f"# TYPE {fam} {kind}\n") == 1 and text.count(f"# HELP {fam} ") == 1
    assert 'stage="say \\"hi\\"\\n"' in text
