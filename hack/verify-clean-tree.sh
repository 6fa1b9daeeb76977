#!/usr/bin/env bash
# CI guard: building and testing must not modify tracked files.
set -euo pipefail
if ! git diff --quiet; then
  git --no-pager diff --stat
  echo "Error: the build/test step modified tracked files" >&2
  exit 1
fi
