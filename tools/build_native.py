#!/usr/bin/env python3
"""Build tritondl's native extensions in-tree (no pip, no JIT cache).

* ``tritondl/_hash_host*.so``  – g++  (OpenSSL EVP host hashing, pybind11)
* ``tritondl/_gpu_hash*.so``   – hipcc --offload-arch=gfx950 (HIP kernels)
* ``tritondl/_relay*.so``      – g++  (native fetch -> S3 data plane + OpenSSL TLS streams, pybind11)
* ``tritondl/_utp*.so``        – g++  (uTP / LEDBAT transport, pybind11)
* ``tritondl/_btwire*.so``     – g++  (BitTorrent peer-wire parser + block assembly, pybind11)

Rebuilds only when a source is newer than its output.  ``--force`` rebuilds.
Cross-compiles fine without a GPU (hipcc needs no device).
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tritondl")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


TARGETS = {
    "_hash_host": {
        "srcs": ["csrc/hash/hash_host.cpp"],
        "cc": "g++",
        "flags": ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", "-Wall"],
        "libs": ["-lcrypto"],
    },
    "_gpu_hash": {
        "srcs": ["csrc/hip/gpu_hash.hip"],
        "deps": ["csrc/hash/hash_core.h"],
        "cc": "hipcc",
        "flags": ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-fvisibility=hidden",
                  "-pthread", "-Wno-unused-result"],
        "libs": ["-lcrypto"],
    },
    "_relay": {
        "srcs": ["csrc/relay/relay.cpp"],
        "deps": ["csrc/hash/hash_core.h"],
        "cc": "g++",
        "flags": ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", "-Wall"],
        "libs": ["-lssl", "-lcrypto"],
    },
    "_btwire": {
        "srcs": ["csrc/btwire/btwire.cpp"],
        "cc": "g++",
        "flags": ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", "-Wall"],
        "libs": [],
    },
    "_utp": {
        "srcs": ["csrc/utp/utp.cpp"],
        "cc": "g++",
        "flags": ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", "-Wall"],
        "libs": [],
    },
}


def out_path(name: str) -> str:
    return os.path.join(PKG, name + _ext_suffix())


def needs_build(name: str, force: bool) -> bool:
    out = out_path(name)
    if force or not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    spec = TARGETS[name]
    deps = [os.path.join(ROOT, s) for s in spec["srcs"] + spec.get("deps", [])]
    for s in spec["srcs"]:
        d = os.path.dirname(os.path.join(ROOT, s))
        deps += [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".cuh"))]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_one(name: str, force: bool = False, verbose: bool = False) -> str:
    spec = TARGETS[name]
    srcs = [os.path.join(ROOT, s) for s in spec["srcs"]]
    if not all(os.path.exists(s) for s in srcs):
        raise FileNotFoundError(f"{name}: missing sources {spec['srcs']}")
    out = out_path(name)
    if not needs_build(name, force):
        return out
    cc = _hipcc() if spec["cc"] == "hipcc" else spec["cc"]
    tmp = out + ".tmp"
    cmd = [cc, *spec["flags"], *_py_includes(), *srcs, "-o", tmp, *spec["libs"]]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build of {name} failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = False, only: list[str] | None = None) -> list[str]:
    outs = []
    for name in TARGETS:
        if only and name not in only:
            continue
        spec = TARGETS[name]
        if not all(os.path.exists(os.path.join(ROOT, s)) for s in spec["srcs"]):
            continue  # component not written yet
        outs.append(build_one(name, force, verbose))
    return outs


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("only", nargs="*")
    a = ap.parse_args()
    for o in build_all(a.force, a.verbose, a.only or None):
        print(o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
