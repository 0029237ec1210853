#!/usr/bin/env python3
"""tools/kres.py K [FILTER] [EXTRA FLAGS...] -- per-kernel resource use (VGPRs, scratch, SGPR / VGPR
spills, occupancy) of the fast march object for depth lanes K, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks; FILTER: a substring of the demangled template
arguments (e.g. "4, 2, true")."""
import re
import subprocess
import sys

K = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
       "-fno-slp-vectorize", "-DVR_MARCH_FAST=1", f"-DVR_MARCH_K={K}", "--offload-device-only", "-c", "vr_march.hip",
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, cwd=__file__.rsplit("/tools/", 1)[0] + "/volume_renderer_amd/csrc", capture_output=True,
                     text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        mg = re.search(r"march_kernelI(.*?)EEv", m.group(1))
        args = re.findall(r"L([ib])(\d+)E", mg.group(1)) if mg else []
        dm = "march_kernel<" + ", ".join(v if t == "i" else ("true" if v == "1" else "false") for t, v in args) + ">" \
            if mg else m.group(1)
        cur = {"name": dm}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+(?:\[[^\]]*\])?):\s+(\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if "march_kernel" in r["name"] and flt in r["name"]:
        args = r["name"].split("march_kernel<", 1)[1].split(">")[0]
        print(f"<{args}>  vgpr {r.get('VGPRs')}  scratch {r.get('ScratchSize [bytes/lane]')}  sgpr_spill "
              f"{r.get('SGPRs Spill')}  vgpr_spill {r.get('VGPRs Spill')}  occ {r.get('Occupancy [waves/SIMD]')}")
