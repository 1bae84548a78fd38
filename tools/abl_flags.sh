#!/bin/bash
# A/B build of the current tree with extra flags on EVERY object (host and
# device: for knobs the host's image / set builds share with the probes, such
# as the hash A/Bs of usn_internal.h): build/abl/<name>/libusn.so.
#   usage: bash tools/abl_flags.sh <name> [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p "build/abl/$name"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
H=/opt/rocm/bin/hipcc
C=usnetd_amd/csrc
$H $F "$@" -c -o build/abl/$name/dev.o $C/usn_device.hip &
$H $F -DUSN_NTHREADS=512 -DUSN_NS=usn_t512 "$@" -c -o build/abl/$name/dev512.o $C/usn_device.hip &
$H $F -DUSN_TEST_HOOKS=1 "$@" -x hip -c -o build/abl/$name/host.o $C/usn_host.cpp &
wait
$H $F -shared -o build/abl/$name/libusn.so build/abl/$name/dev.o build/abl/$name/dev512.o build/abl/$name/host.o
echo "built build/abl/$name/libusn.so ($*)"
