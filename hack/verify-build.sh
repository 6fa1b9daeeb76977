#!/usr/bin/env bash
# Rebuild every native extension from scratch and import the package:
# fails if a source no longer compiles for gfx950 or a module does not load.
set -euo pipefail
cd "$(dirname "$0")/.."
python3 tools/build_native.py --force -v
python3 -c "import tritondl.ops.hashing as h, tritondl.fetch.bt.utp, tritondl.service; h.gpu_module(); print('native OK')"
