#!/bin/bash
# Check out an old commit as a separate tree for a box A/B, instead of
# copying old sources over the working tree (a box script must never
# overwrite tracked files).  The tree lands in .ab/<name> (git-ignored, but
# NOT gpurun-ignored, so it travels with the snapshot; the box has no .git),
# with this tree's built native modules copied in.  Usage:
#   tools/ab_tree.sh <commit> <name>     then on the box: (cd .ab/<name> && python bench.py ...)
#   tools/ab_tree.sh --build <commit> <name>   build that commit's own native modules instead of
#                                              copying this tree's (an A/B of native code)
#   tools/ab_tree.sh --remove <name>
set -euo pipefail
cd "$(git rev-parse --show-toplevel)"
if [ "${1:-}" = "--remove" ]; then
  git worktree remove --force ".ab/$2"
  exit 0
fi
build=0
if [ "${1:-}" = "--build" ]; then build=1; shift; fi
commit=$1 name=$2
mkdir -p .ab
git worktree add --force --detach ".ab/$name" "$commit" >/dev/null
if [ $build = 1 ]; then
  (cd ".ab/$name" && python tools/build_native.py >/dev/null)
else
  cp tritondl/*.so ".ab/$name/tritondl/"
fi
echo ".ab/$name @ $(git rev-parse --short "$commit")"
