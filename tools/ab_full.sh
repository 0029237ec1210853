#!/bin/bash
# tools/ab_full.sh NAME "EXTRA FLAGS" -- like tools/ab_tree.sh, but every object is rebuilt with the
# flags (for switches the host code reads too, e.g. VR_PROBE_MAX in vr_device.h).
set -e
cd "$(dirname "$0")/.."
S=build_ab/src_$1
rm -rf $S && mkdir -p $S/volume_renderer_amd
cp -rp volume_renderer_amd/csrc $S/volume_renderer_amd/ && cp -rp include $S/
rm -f $S/volume_renderer_amd/csrc/*.o
make -s -j8 -C $S/volume_renderer_amd/csrc OUT="$PWD/build_ab/libvrhip_$1.so" EXTRA="$2" 2>&1 | grep -E "error|Error" || true
rm -rf $S
ls -la build_ab/libvrhip_$1.so
