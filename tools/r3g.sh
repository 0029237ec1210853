#!/bin/bash
# round-3 pass g: exact cosines in the fast variant (cos0) -- same-box A/B and full-size parity --
# then the measurement pass of the default library: bench line, kernel trace, PMC passes
RUN=${1:-r3g}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 2 "tree=VR_X=1" "cos0=VR_LIB_PATH=build_ab/libvrhip_cos0.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
" > gpurun_out/$RUN/ab.txt && cat gpurun_out/$RUN/ab.txt &&
ABL_SCENES=c2,metric,c4_main timeout -k 10 900 python -u tools/shade_ablation.py gpurun_out/$RUN/ablation.json \
  base=default cos0=build_ab/libvrhip_cos0.so exact=default:VR_EXACT_SHADE=1 > gpurun_out/$RUN/ablation.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err &&
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$RUN/kt -o kt --output-format csv -- \
   python bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipelined-streams 0 > gpurun_out/$RUN/kt.log 2>&1) &&
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum,TCC_MISS_sum,TCC_REQ_sum;SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SMEM;SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE;GRBM_GUI_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_THREAD_CYCLES_VALU" \
  bash tools/pmc.sh gpurun_out/$RUN/pmc &&
cat gpurun_out/$RUN/bench.json
