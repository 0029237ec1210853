#!/usr/bin/env python3
"""tools/isa_hot.py [ASM] -- instruction classes on the common path of the production march kernel's
sample loop (/tmp/probe.s from tools/isa_probe.sh): the fast (tame, finite) copy's depth-2 loop that
holds the depth-lane compositing (v_mov_b32_dpp), minus the blocks of the global-memory fallbacks
(64-bit addressing: v_lshl_add_u64 / v_mad_u64_u32) and of NaN-checking code.  A static estimate of
one lit wave-iteration, for comparing builds."""
import collections
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "/tmp/probe.s"
s = open(path).read()
name = re.search(r"(_ZN2vr4fast12march_kernelILi2ELi1ELb1ELb0ELb1ELb0ELi(?:1664|2040)ELi0E(?:Li\d+E)?EEvNS_12RenderParamsE):", s).group(1)
body = s[s.index(name + ":"):s.index(".Lfunc_end", s.index(name + ":"))].split("\n")
blocks, cur = [], None
for l in body:
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", l) or re.match(r"^; %bb\.(\d+):(.*)", l)
    if m:
        cur = {"name": m.group(1), "hdr": m.group(2), "ins": []}
        blocks.append(cur)
        continue
    t = l.strip()
    if cur is None or not t or t.startswith((".", ";")):
        continue
    cur["ins"].append(t.split(";")[0].strip())
# loop headers named in the comments: 'Loop: Header=BBx_y Depth=2'
dpp = [i for i, b in enumerate(blocks) if any(x.startswith("v_mov_b32_dpp") and "quad_perm" in x for x in b["ins"])]
hdrs = []
for i in dpp:
    m = re.search(r"Header=BB(\d+_\d+) Depth=2", blocks[i]["hdr"])
    if m and m.group(1) not in hdrs:
        hdrs.append(m.group(1))
# the tame (NANCHK = false) copy: the sample loop without NaN checks (v_cmp_o_f32)
best = None
for h in hdrs:
    lp = [b for b in blocks if f"Header=BB{h} " in b["hdr"] or b["name"] == f".LBB{h}"]
    nan = sum(1 for b in lp for x in b["ins"] if x.startswith("v_cmp_o_f32"))
    if best is None or nan < best[1]:
        best = (h, nan, lp)
hdr, _, loop = best
hot = [b for b in loop if not any(x.startswith(("v_lshl_add_u64", "v_mad_u64_u32")) for x in b["ins"])]
# the lights past the first pair (held in registers since round 4) are loaded by index inside the loop:
# their blocks are off the common path of a two-light frame (--all keeps them)
if "--all" not in sys.argv:
    hot = [b for b in hot if not any(x.startswith("s_load_") for x in b["ins"])]
c = collections.Counter(x.split()[0] for b in hot for x in b["ins"])
valu = sum(n for k, n in c.items() if k.startswith("v_"))
slow = sum(n for k, n in c.items() if k.startswith(("v_cmp", "v_cvt", "v_floor", "v_rndne", "v_fract", "v_med3",
                                                     "v_max_i", "v_min_i", "v_mul_lo", "v_mad_u32", "v_add3",
                                                     "v_readlane", "v_writelane")))
trans = sum(n for k, n in c.items() if k.startswith(("v_rsq", "v_sqrt", "v_exp", "v_rcp", "v_log")))
print(f"loop BB{hdr}: {len(loop)} blocks, common path {len(hot)}: instructions {sum(c.values())}, VALU {valu} "
      f"(slow class {slow}, transcendental {trans}), readlane {c['v_readlane_b32']}, s_nop {c['s_nop']}, "
      f"scratch {c['scratch_load_dword'] + c['scratch_load_dwordx2']}, LDS {sum(n for k, n in c.items() if k.startswith('ds_'))}")
if "--dump" in sys.argv:
    for b in hot:
        print(b["name"], b["hdr"][:80])
        for x in b["ins"]:
            print("   ", x)
