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


def test_shared_native_headers_link_into_two_translation_units():
    """Every csrc header is safe to include from more than one TU."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "odr_check.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_product_package_does_not_ship_or_import_the_harness():
    """The fakes, bench drivers and soak live in tritondl_testkit, outside the
    wheel (pyproject) and the image (Dockerfile copies tritondl/ only), and
    the worker never imports them."""
    import subprocess
    import sys
    code = ("import sys, tritondl.service, tritondl.parallel.pool, tritondl.check; "
            "print([m for m in sys.modules if m.startswith('tritondl_testkit')])")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[]", r.stdout
    assert not os.path.exists(os.path.join(ROOT, "tritondl", "fakes"))
    for f in ("bench_job.py", "bench_producer.py", "soak.py"):
        assert not os.path.exists(os.path.join(ROOT, "tritondl", f))
    py = open(os.path.join(ROOT, "pyproject.toml")).read()
    assert 'include = ["tritondl", "tritondl.*"]' in py
    df = open(os.path.join(ROOT, "docker", "Dockerfile")).read()
    assert "COPY --from=build /src/tritondl/tritondl /app/tritondl" in df and "tritondl_testkit" in df


def test_lint_clean():
    """tools/lint.py (compile + unused imports, standard library only) finds nothing."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "tools", "lint.py")], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
