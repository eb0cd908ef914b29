#!/bin/bash
# Build an experimental libhorreum_gpu.so with extra defines into build_exp/<name>/
# (git-ignored; travels to the GPU box).  Usage: tools/build_variant.sh NAME "-DFOO=1 ..."
set -e
name=$1; defs=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build_exp/$name
rm -rf "$out"; mkdir -p "$out"
cd "$root/horreum_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-value -Wno-unused-result $defs"
pids=()
for f in hg_decode hg_encode hg_merge hg_lookup hg_runtime hg_multi; do
  /opt/rocm/bin/hipcc $F -c $f.hip -o "$out/$f.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o "$out/libhorreum_gpu.so" "$out"/*.o
echo "$out/libhorreum_gpu.so"
