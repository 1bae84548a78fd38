#!/bin/bash
# A/B build of an earlier commit's library: build/abl/<name>/libusn.so from
# the C sources of <commit> (same compiler flags as the Makefile), so that
# tools/abl.py and tools/scatter_bench.py time it beside the current tree in
# one process.   usage: bash tools/abl_commit.sh <name> <commit> [extra hipcc flags]
set -e
name=$1; commit=$2; shift 2
src=build/abl_src/$name
rm -rf "$src"; mkdir -p "$src" "build/abl/$name"
git archive "$commit" usnetd_amd/csrc include | tar -x -C "$src"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
H=/opt/rocm/bin/hipcc
$H $F -DUSN_AB_BUILD=1 "$@" -c -o build/abl/$name/dev.o $src/usnetd_amd/csrc/usn_device.hip &
$H $F -DUSN_AB_BUILD=1 -DUSN_NTHREADS=512 -DUSN_NS=usn_t512 "$@" -c -o build/abl/$name/dev512.o $src/usnetd_amd/csrc/usn_device.hip &
$H $F -x hip -c -o build/abl/$name/host.o $src/usnetd_amd/csrc/usn_host.cpp &
wait
$H $F -shared -o build/abl/$name/libusn.so build/abl/$name/dev.o build/abl/$name/dev512.o build/abl/$name/host.o
echo "built build/abl/$name/libusn.so from $commit"
