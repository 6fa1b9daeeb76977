"""Dev tooling (reference C16: ``hack/load-env.sh``, ``modd.conf``,
``renovate.json``, ``CODEOWNERS``)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_load_env_exports_every_assignment(tmp_path):
    """``. hack/load-env.sh FILE`` exports KEY=VALUE lines, skipping comments
    and blanks, like the reference's ``hack/load-env.sh``; a missing file is
    an error."""
    env_file = tmp_path / ".env"
    env_file.write_text("# broker\nRABBITMQ_ENDPOINT=10.0.0.5:5672\n\n  # indented comment\n"
                        "S3_ENDPOINT=http://minio:9000\nLOG_FORMAT=json\n")
    script = (f". {ROOT}/hack/load-env.sh {env_file} >/dev/null && "
              "python3 -c 'import os; print(os.environ[\"RABBITMQ_ENDPOINT\"], os.environ[\"S3_ENDPOINT\"], "
              "os.environ[\"LOG_FORMAT\"])'")
    p = subprocess.run(["bash", "-c", script], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["10.0.0.5:5672", "http://minio:9000", "json"]
    p = subprocess.run(["bash", "-c", f". {ROOT}/hack/load-env.sh {tmp_path}/missing"], capture_output=True,
                       text=True, timeout=30)
    assert p.returncode != 0 and "no env file" in p.stderr


def test_devwatch_sees_python_and_native_changes(tmp_path):
    """``tools/devwatch.py`` (the reference's ``modd.conf``) watches the Python
    package and the native sources."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import devwatch
    finally:
        sys.path.pop(0)
    snap = devwatch.snapshot()
    assert any(p.endswith(os.path.join("tritondl", "service.py")) for p in snap)
    assert any(p.endswith(".hip") for p in snap) and any(p.endswith(".cpp") for p in snap)


def test_repo_metadata_is_valid():
    with open(os.path.join(ROOT, "renovate.json")) as f:
        cfg = json.load(f)
    assert "pep621" in cfg["enabledManagers"]
    with open(os.path.join(ROOT, ".github", "CODEOWNERS")) as f:
        rules = [ln.split() for ln in f if ln.strip() and not ln.startswith("#")]
    assert rules and all(len(r) >= 2 and r[1].startswith("@") for r in rules)
