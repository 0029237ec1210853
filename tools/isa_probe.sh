#!/bin/bash
# tools/isa_probe.sh [EXTRA_FLAGS] -- compile only the metric frame's production march kernel
# (fast shading, K = 2, half-texel taps, 32-bit, 6.5 KiB slots, unscheduled) to /tmp/probe.s and
# print its resource use and the instruction classes that cost issue slots.
cd "$(dirname "$0")/../volume_renderer_amd/csrc"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
  -DVR_MARCH_FAST=1 -DVR_MARCH_K=2 -DVR_ISA_PROBE=1 $1 --offload-device-only -S vr_march.hip -o /tmp/probe.s || exit 1
python3 - <<'PY'
import re, collections
s = open('/tmp/probe.s').read()
name = re.search(r'(_ZN2vr4fast12march_kernelILi2ELi1ELb1ELb0ELb1ELb0ELi(?:1664|2040)ELi0E(?:Li\d+E)?EEvNS_12RenderParamsE):', s).group(1)
body = s[s.index(name + ':'):s.index('.Lfunc_end', s.index(name + ':'))]
ins = [l.strip().split()[0] for l in body.split('\n') if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':')]
c = collections.Counter(ins)
meta = s[s.index('.amdhsa_kernel ' + name):]
g = lambda k: re.search(k + r' (\d+)', meta).group(1)
print('instructions', len(ins), 'vgpr', g('.amdhsa_next_free_vgpr'), 'sgpr', g('.amdhsa_next_free_sgpr'),
      'scratch', g('.amdhsa_private_segment_fixed_size'))
for k in ('v_readlane_b32', 'v_writelane_b32', 's_nop', 'scratch_load_dword', 'scratch_load_dwordx2', 'v_mov_b32_dpp',
          'v_mul_lo_u32', 'v_cvt_i32_f32_e32', 'v_cmp_gt_u32_e32', 'v_cndmask_b32_e64'):
    print(f'  {k:24s} {c.get(k, 0)}')
PY
