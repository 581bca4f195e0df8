#!/bin/bash
# Build libpbn_env.so of a git revision (default HEAD) into pbn_rl_amd/libpbn_env_diag_base.so,
# the "before" side of an A/B run (tools/chunk_fit.py with PBN_LIB=...).
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" pbn_rl_amd/csrc include | tar -x -C "$TMP"
srcs=("$TMP"/pbn_rl_amd/csrc/*.hip)   # every translation unit of that revision
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result \
  -o "$ROOT/pbn_rl_amd/libpbn_env_diag_base.so" "${srcs[@]}"
rm -rf "$TMP"
echo "built $REV -> pbn_rl_amd/libpbn_env_diag_base.so"
