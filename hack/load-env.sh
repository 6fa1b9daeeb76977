#!/usr/bin/env bash
# Source me: export every KEY=VALUE line of ./.env (comments and blanks skipped).
#   . hack/load-env.sh [path/to/.env]
f="${1:-.env}"
if [[ ! -f "$f" ]]; then echo "no env file '$f'" >&2; return 1 2>/dev/null || exit 1; fi
echo "loading env variables from '$f'"
set -a
# shellcheck disable=SC1090
. <(grep -Ev '^\s*(#|$)' "$f")
set +a
