#!/bin/bash
# tools/ab_tree.sh NAME "EXTRA FLAGS" -- build libvrhip.so of the working tree with extra compiler
# flags into build_ab/libvrhip_NAME.so for a same-box A/B (VR_LIB_PATH=...).  The in-tree objects
# are reused (timestamps kept) except the fast march objects, which the flags are meant for.
set -e
cd "$(dirname "$0")/.."
S=build_ab/src_$1
rm -rf $S && mkdir -p $S/volume_renderer_amd
cp -rp volume_renderer_amd/csrc $S/volume_renderer_amd/ && cp -rp include $S/
rm -f $S/volume_renderer_amd/csrc/vr_march_fast_k*.o
make -s -j8 -C $S/volume_renderer_amd/csrc OUT="$PWD/build_ab/libvrhip_$1.so" EXTRA="$2" 2>&1 | grep -E "error|Error" || true
rm -rf $S
ls -la build_ab/libvrhip_$1.so
