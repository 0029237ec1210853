#!/usr/bin/env python3
"""tools/gpupass.py RUN STEP [STEP ...] -- one measurement pass on the GPU box (run through gpurun).

Replaces the per-pass shell scripts of rounds 1-3: a pass is a list of steps, each run in a child
process with its own time limit, output under gpurun_out/RUN/; the pass stops at the first step
that fails (a GPU fault, an abort or a time limit ends the call -- nothing is retried).

Steps ('|' separates variants, ',' environment assignments inside a variant):
  tests[:K_EXPR]                 pytest -m gpu (optionally -k K_EXPR)            -> tests.log
  ab:ROUNDS:NAME=ENV,..|NAME=..  interleaved same-box bench.py A/B (serial frames, 20 steps); a
                                 variant's ENV may hold VR_LIB_PATH=build_ab/libvrhip_X.so; extra
                                 bench args from the last args: step    -> abN.jsonl, abN.txt (N-th ab)
  args:BENCH_ARGS                bench.py arguments of the following ab steps (e.g. --width 1024
                                 --height 768; '-' for none)
  abl:SCENES:NAME=LIB[;ENV,..]|..  tools/shade_ablation.py parity of shading variants on the scenes
                                 (c2, metric, c4_main, c4_struct)                  -> ablation.json
  bench[:ARGS]                   the bench line (CPU baseline included unless ARGS say otherwise)
                                 -> bench.json (the N-th bench step of a pass: benchN.json)
  kt[:ARGS]                      rocprofv3 --kernel-trace --stats of bench.py      -> ktN/ (N-th kt)
  pmc[:[@K=V,..@]ARGS]           tools/pmc.sh counter passes (one group per pass)  -> pmcN/ (N-th pmc);
                                 @..@ sets the environment (e.g. VR_LIB_PATH of a variant)
  py:SCRIPT[ ARGS]               any python script of the tree (e.g. tools/tail_profile.py ...)
"""
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def run(cmd, log, limit, env=None):
    t0 = time.time()
    with open(log, "ab") as fh:
        fh.write(("$ " + " ".join(cmd) + "\n").encode())
        fh.flush()
        rc = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, cwd=ROOT, stdout=fh, stderr=subprocess.STDOUT,
                            env=env).returncode
    print(f"  [{time.time() - t0:6.1f} s] rc={rc} {' '.join(cmd)[:140]}", flush=True)
    return rc


def parse_env(spec):
    env = {}
    for kv in spec.split(","):
        if kv and kv != "-":
            k, v = kv.split("=", 1)
            env[k] = v
    return env


def step_ab(out, rest, idx, bench_args):
    rounds, variants = rest.split(":", 1)
    specs = []
    for v in variants.split("|"):
        name, _, envs = v.partition("=")
        specs.append((name, parse_env(envs)))
    jl = os.path.join(out, f"ab{idx}.jsonl")
    extra = shlex.split(bench_args)
    for r in range(int(rounds)):
        for name, env in specs:
            e = dict(os.environ, VR_TEST_SWITCHES="1")  # (bench.py: the library reads the VR_* switches)
            e.update(env)
            res = os.path.join(out, f"ab{idx}_{name}_{r}.json")
            cmd = [PY, "bench.py", "--steps", "20", "--warmup", "4", "--no-cpu-baseline", "--pipelined-streams", "0"]
            with open(res, "wb") as fh:
                rc = subprocess.run(["timeout", "-k", "10", "300"] + cmd + extra, cwd=ROOT, stdout=fh,
                                    stderr=subprocess.DEVNULL, env=e).returncode
            if rc:
                print(f"  ab {name} round {r}: rc={rc}")
                return rc
            line = json.loads(open(res).read().strip().splitlines()[-1])
            with open(jl, "a") as fh:
                fh.write(json.dumps({"ab": name, "round": r, "args": bench_args, "line": line}) + "\n")
            rf = line.get("roofline", {})
            print(f"  ab {name:10s} round {r}: frame {line['ms_per_step']:.3f} ms, kernel {rf.get('kernel_ms')} ms, "
                  f"sha {str(line.get('image_sha256', ''))[:12]}", flush=True)
    summary = {}
    for l in open(jl):
        d = json.loads(l)
        summary.setdefault(d["ab"], []).append(d["line"]["roofline"].get("kernel_ms"))
    with open(os.path.join(out, f"ab{idx}.txt"), "w") as fh:
        fh.write(f"bench args: {bench_args or '(default)'}\n")
        for k, v in summary.items():
            fh.write(f"{k} {v} min {min(v)}\n")
    return 0


def main():
    run_name, steps = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "gpurun_out", run_name)
    os.makedirs(out, exist_ok=True)
    n_ab, n_kt, n_pmc, n_bench, bench_args = 0, 0, 0, 0, ""
    for st in steps:
        kind, _, rest = st.partition(":")
        print(f"step {kind}: {rest[:120]}", flush=True)
        if kind == "tests":
            # -rP: the captured output of passed tests too (the PARITY lines of test_full_size.py,
            # tools/parity_summary.py)
            cmd = [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-v", "-rP", "--timeout", "120",
                   "--timeout-method", "thread"] + (["-k", rest] if rest else [])
            rc = run(cmd, os.path.join(out, "tests.log"), 900)
        elif kind == "ab":
            n_ab += 1
            rc = step_ab(out, rest, n_ab, bench_args)
        elif kind == "args":
            bench_args = "" if rest == "-" else rest
            rc = 0
        elif kind == "abl":
            scenes, variants = rest.split(":", 1)
            args = [v.replace(";", ":", 1) for v in variants.split("|")]
            e = dict(os.environ, ABL_SCENES=scenes)
            rc = run([PY, "-u", "tools/shade_ablation.py", os.path.join(out, "ablation.json")] + args,
                     os.path.join(out, "ablation.log"), 1100, env=e)
        elif kind == "bench":
            n_bench += 1
            tag = "bench" if n_bench == 1 else f"bench{n_bench}"
            with open(os.path.join(out, tag + ".json"), "wb") as fh, open(os.path.join(out, tag + ".err"), "wb") as fe:
                rc = subprocess.run(["timeout", "-k", "10", "500", PY, "bench.py"] + shlex.split(rest), cwd=ROOT,
                                    stdout=fh, stderr=fe).returncode
            print(f"  {tag} rc={rc} ({rest or 'default'})", flush=True)
        elif kind == "kt":
            args = shlex.split(rest) or ["--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--pipelined-streams",
                                         "0"]
            e = dict(os.environ, TMPDIR="/tmp")
            n_kt += 1
            rc = run(["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(out, f"kt{n_kt}"), "-o", "kt",
                      "--output-format", "csv", "--", PY, "bench.py"] + args, os.path.join(out, f"kt{n_kt}.log"), 400,
                     env=e)
        elif kind == "pmc":
            n_pmc += 1
            penv = None
            if rest.startswith("@"):  # pmc:@K=V,K=V@ ARGS -- environment of the profiled runs
                spec, _, rest = rest[1:].partition("@")
                penv = dict(os.environ)
                penv.update(parse_env(spec))
            rc = run(["bash", "tools/pmc.sh", os.path.join(out, f"pmc{n_pmc}")] + shlex.split(rest),
                     os.path.join(out, f"pmc{n_pmc}.log"), 1000, env=penv)
        elif kind == "py":
            rc = run([PY, "-u"] + shlex.split(rest), os.path.join(out, "py.log"), 900)
        else:
            print(f"unknown step {kind}")
            rc = 2
        if rc:
            print(f"pass {run_name}: step {kind} failed (rc {rc}); stopping")
            return rc
    print(f"pass {run_name}: done")
    return 0


if __name__ == "__main__":
    sys.exit(main())
