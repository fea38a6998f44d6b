#!/bin/bash
# Build the HIP library of a git revision (or the working tree: REV=WORK) into exp/NAME/libdofs_hip.so, for the
# same-box A/B scripts (tools/ab.sh, tools/ab_env.sh). Usage: bash tools/build_variant.sh NAME [REV] [extra hipcc flags]
set -eu
name=$1; rev=${2:-WORK}; shift 2 || true
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/exp/src_$name
rm -rf "$src"; mkdir -p "$src/csrc" "$root/exp/$name"
ln -sfn "$root/include" "$root/exp/include"
if [ "$rev" = WORK ]; then
    cp "$root"/denseopticalflowsegmentation3d_amd/csrc/*.{h,hip} "$src/csrc/"
else
    for f in $(git -C "$root" ls-tree --name-only "$rev" denseopticalflowsegmentation3d_amd/csrc/); do
        case $f in *.h|*.hip) git -C "$root" show "$rev:$f" > "$src/csrc/$(basename "$f")" ;; esac
    done
fi
# exp/src_NAME/csrc/../../include = exp/include -> the repo's include/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result "$@" -shared \
    -o "$root/exp/$name/libdofs_hip.so" "$src/csrc/dofs_hip.hip"
echo "exp/$name/libdofs_hip.so <- $rev"
