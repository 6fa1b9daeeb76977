#!/usr/bin/env bash
# Run the CI "cpu" job's steps (.github/workflows/ci.yml) in this checkout,
# without the pip step (the image has every dependency): rebuild + import,
# lint, CPU test suite, native self-test under ASan/UBSan and TSan, ODR link
# check, clean tree.
set -euo pipefail
cd "$(dirname "$0")/.."
step() { echo "=== $* ($(date -u +%H:%M:%S))"; "$@"; }
step ./hack/verify-build.sh
step python3 tools/lint.py
step python3 -m pytest tests -x -q -m "not gpu" -n 4 --timeout 600
step python3 tools/native_selftest.py --sanitize
step python3 tools/odr_check.py
step ./hack/verify-clean-tree.sh
echo "=== CI cpu job OK"
