#!/bin/bash
# tools/ab_rev.sh NAME REV [make flags] -- build libvrhip.so of git revision REV (committed sources
# only) into build_ab/libvrhip_NAME.so for an A/B run on the GPU box (VR_LIB_PATH=...).
set -e
cd "$(dirname "$0")/.."
rm -rf build_ab/src_$1 && mkdir -p build_ab/src_$1
git archive "$2" volume_renderer_amd/csrc include | tar -x -C build_ab/src_$1
make -s -j8 -C build_ab/src_$1/volume_renderer_amd/csrc OUT="$PWD/build_ab/libvrhip_$1.so" "${@:3}"
rm -rf build_ab/src_$1
ls -la build_ab/libvrhip_$1.so
