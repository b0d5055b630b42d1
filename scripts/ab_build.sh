#!/bin/bash
# Side build for same-box A/B runs: copy the tree into ab/<name> and rebuild every HIP object with
# extra compiler flags (e.g. -DDL_GEMV_RING=8). ab/ is git-ignored; it travels with gpurun while it
# exists (delete it after the A/B).  usage: scripts/ab_build.sh <name> "<EXTRA_HIPFLAGS>" [-jN]
set -e
name=$1; flags=$2; jobs=${3:--j8}
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/ab/$name
mkdir -p "$dst"
rm -rf "$dst"; mkdir -p "$dst"
(cd "$root" && tar cf - --exclude ./.git --exclude ./ab --exclude ./gpurun_out --exclude './BENCH_*' \
  --exclude './GPUTEST_*' --exclude ./profiles --exclude '__pycache__' .) | (cd "$dst" && tar xf -)
rm -rf "$dst/build/obj/hip"
make -C "$dst" $jobs all EXTRA_HIPFLAGS="$flags" > "$dst/build.log" 2>&1 || { tail -20 "$dst/build.log"; exit 1; }
echo "built ab/$name with $flags"
