"""Benchmark: env-steps/s of T1DHStandEnv.step() (the LeggedRobot.step() hot path) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--num-envs 8192] [--mesh trimesh]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], the metric's config): t1_dh_stand, 8192 envs per GPU, trimesh
curriculum terrain (20 x 20 sub-terrains) + the full DHT1StandCfg domain randomisation, synthetic
random-command rollouts: actions ~ N(0, 1) pre-generated on the device (policy inference excluded), the
env's own gait scheduler draws the commands.  One step = one env.step(actions) for all envs on the rank
(10 physics substeps + post-physics + 66-frame obs stack).  N > 1: envs shard by global env id across the
ranks (weak scaling; the env step has no collective), timed region bracketed by barrier + synchronize,
max over ranks.

roofline: SURVEY.md §8(d): achieved = env_steps_per_s x B_alg (30,678 algorithmic bytes per env-step) against
the 8 TB/s HBM3E peak; `traffic` = PMC-measured HBM bytes per step (profiles/traffic_*.json, tools/
pmc_traffic.py).  Per-kernel durations are measured live with HIP events around each launch on every
--time-every'th timed step (event records cost host time, so not on every step), with each kernel's own
algorithmic bytes; the dominant kernel is the whole fused step -- k_dyn6 (eight role waves, two per SIMD; latency-bound
on its core wave's chain) at every config but config 5's fp16 histories, where t1env picks k_dyn4 with its
history shift as a concurrent launch (fused_kernel below names the kernel of each run).
cpu_baseline: the build's CPU restatement (numpy oracle post-physics + OpenMP dynamics), rank 0, N = 1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

B_ALG = 30678          # algorithmic bytes per env-step (fp32, default t1 config)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SHADER_GHZ = 2.4       # MI355X peak engine clock
# the committed PMC traffic profiles (tools/pmc_traffic.py over rocprofv3 FETCH_SIZE / WRITE_SIZE passes): config 3
# (the metric) and config 5; the roofline's "traffic" is the one whose workload matches the run's, else null
TRAFFIC_PROFILES = [os.path.join(REPO, "profiles", f) for f in ("traffic_r07fb.json", "traffic_r07fb_cfg5.json")]
LONE_WAVE_VALU_PER_CYCLE = 0.25  # one VALU instruction per 4 cycles for a wave alone on its SIMD (MI355X_MICROARCH.md,
                                 # 'vector-instruction ISSUE cost'); k_dyn5 runs one wave per SIMD (405 registers)
SIMD_VALU_PER_CYCLE = 0.5        # a SIMD with two or more waves: one wave64 VALU instruction per 2 cycles (k_dyn6)
# timer slots of include/t1env.h: slot "k_dynamics" brackets the dynamics launch, which on a normal step is the
# whole fused step (k_dyn6: dynamics + in-workgroup history shift + post-physics epilogue, t1env_dyn6.hip);
# k_post_a / k_post_b only launch on the split (command-curriculum, 1 in 2400) steps
KERNELS = ["k_dynamics", "k_post_a", "k_post_b"]
def fused_kernel(num_envs, cus=256, obs_half=False):
    """The step kernel t1env picks (t1_dyn_waves_default): k_dyn6, k_dyn4 for fp16 histories above one round of 32-env
    workgroups; the T1ENV_DYN_KERNEL override wins."""
    k = os.environ.get("T1ENV_DYN_KERNEL")
    if k in ("4", "5", "6"):
        return "k_dyn" + k
    return "k_dyn4" if obs_half and (num_envs + 31) // 32 > cus else "k_dyn6"
# per-kernel algorithmic bytes per env (reads + writes it must do) for the split sequence
SHIFT_BYTES = 2 * 4 * ((3102 - 47) + (219 - 73))
KERNEL_BYTES = {
    "k_dynamics": 4 * (13 + 24 + 12 + 48 + 12 * 6 + 13 + 3 + 3) + 4 * (13 + 24 + 169 + 39 + 12 + 12 + 12 + 24 + 6)
    + SHIFT_BYTES,
    "k_post_a": 4 * (13 + 24 + 169 + 39 + 12 * 5 + 6 + 4 + 24 + 12 + 3 + 6 + 8) + 4 * (3 * 4 + 6 + 3 + 2 + 4 + 24 + 3 + 6),
    "k_post_b": 4 * (24 + 13 + 12 * 2 + 3 * 3 + 39 + 24 + 6 + 8) + 4 * (47 + 73 + 12 * 4 + 6),
}


def alg_bytes(state_dtype):
    """(B_alg, history-shift bytes) per env-step: SURVEY.md §8(d)'s 30,678 B with fp32 histories; with fp16 histories
    (config 5) the four history terms (obs write 12,408 + read 12,220, priv write 876 + read 584) halve -> 17,634."""
    if state_dtype == "fp16":
        return B_ALG - (12408 + 12220 + 876 + 584) // 2, SHIFT_BYTES // 2
    return B_ALG, SHIFT_BYTES


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--mesh", default="trimesh", choices=["plane", "heightfield", "trimesh"])
    p.add_argument("--state-dtype", default="fp32", choices=["fp32", "fp16"],
                   help="storage dtype of the obs / critic histories (fp16: BASELINE config 5's fp16 state)")
    p.add_argument("--push", action="store_true", help="domain_rand.push_robots on (BASELINE config 5), every 6 s")
    p.add_argument("--repeats", type=int, default=1,
                   help="time the K steps R times (each bracketed by barrier + synchronize) and report the median "
                        "(SURVEY §8(d): median of 5); the per-repeat values go to repeat_values")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-self-collision", action="store_true",
                   help="A/B only (not the metric's config): asset.self_collisions = 1 (Isaac Gym's filter: disabled)")
    p.add_argument("--time-every", type=int, default=8,
                   help="record per-kernel HIP events on every k-th timed step (event records cost host time; "
                        "0 = never, 1 = every step)")
    p.add_argument("--cpu-envs", type=int, default=None,
                   help="CPU-baseline env count (default: --num-envs, the metric's 8192; VERDICT r4 #7)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--cpu-shards", type=int, default=32,
                   help="CPU baseline: env shards stepped on Python threads (at most the affinity's core count)")
    p.add_argument("--traffic-json", default=None,
                   help="PMC-measured HBM bytes per kernel (from tools/pmc_traffic.py); default: the committed profile "
                        "of this workload (TRAFFIC_PROFILES), included when one matches")
    p.add_argument("--sq-json", default=os.path.join(REPO, "profiles", "r07fb_sq_counters.json"),
                   help="SQ instruction counters of the fused kernel (tools/pmc_sq_summary.py): the VALU-issue roofline")
    return p.parse_args()


def effective_cores():
    """The cores this process can use: its CPU affinity, capped by the cgroup CPU quota.  On the GPU box the affinity
    lists every core of the host (256) while the job's cgroup grants a share of them (cpu.max, e.g. 16): 256 threads
    on a 16-core quota ran the CPU baseline 3.5x slower than 16 (r04fa)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except Exception:
            quota = None
    if quota is not None:
        n = min(n, max(1, int(quota + 0.5)))
    return n


def cpu_baseline(env, args):
    """Bounded sample of the same workload on the host cores (the build's CPU restatement), at the metric's env count
    unless --cpu-envs says otherwise."""
    if args.cpu_envs is None:
        args.cpu_envs = args.num_envs
    from oracle.cpu_env import ShardedCpuT1Env
    terrain = None
    if env.mesh_type in ("heightfield", "trimesh"):
        tc = env.cfg.terrain
        terrain = {"terrain_origins": env._terrain.env_origins, "height_samples": env._terrain.heightsamples,
                   "horizontal_scale": tc.horizontal_scale, "vertical_scale": tc.vertical_scale,
                   "border_size": tc.border_size, "num_envs_total": args.cpu_envs}
    aff = effective_cores()
    # every core this process may run on (not the inherited OMP_NUM_THREADS): shards of the env on
    # Python threads (the numpy post-physics releases the GIL in its array kernels), each with cores / shards OpenMP
    # threads for its physics
    cpu = ShardedCpuT1Env(env._model, args.cpu_envs, cores=aff, shards=min(aff, args.cpu_shards), seed=5,
                          mesh_type=env.mesh_type, terrain=terrain)
    cpu.reset()
    rng = np.random.default_rng(0)
    acts = rng.standard_normal((8, args.cpu_envs, 12)).astype(np.float32)
    cpu.step(acts[0])
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        cpu.step(acts[n % 8])
        n += 1
    dt = time.perf_counter() - t0
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(args.cpu_envs * n / dt, 1), "unit": "env-steps/s", "cores": cpu.threads(), "kind": "port",
            "sample": f"{args.cpu_envs} envs x {n} steps ({dt:.1f} s), same cfg/terrain as the GPU run; "
                      f"{len(cpu.shards)} env shards on Python threads (numpy oracle PD + post-physics) with "
                      f"{cpu.threads() // len(cpu.shards)} OpenMP threads each for the fp32 dynamics: {cpu.threads()} "
                      f"threads on the {aff} cores this process may use (affinity capped by the cgroup CPU quota), {model}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL ("nccl").  T1_BENCH_BACKEND=gloo (tests/test_gpu_bench_multirank.py only): the same
    # N > 1 path with ranks sharing a GPU, which RCCL refuses -- the local rank then wraps around the visible devices
    backend = os.environ.get("T1_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if (backend != "nccl" and ndev > 0) else local
    dev = torch.device(f"cuda:{local_dev}")
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
    torch.cuda.set_device(dev)
    from ti5_isaacgym_amd import make_t1_env
    N = args.num_envs
    def hook(cfg):
        cfg.env.state_dtype = args.state_dtype
        cfg.domain_rand.push_robots = bool(args.push)
        if args.no_self_collision:
            cfg.asset.self_collisions = 1
    env = make_t1_env(num_envs=N, mesh_type=args.mesh, seed=5, device=str(dev), env_offset=rank * N,
                      num_envs_total=N * world, cfg_hook=hook)
    b_alg, shift_bytes = alg_bytes(args.state_dtype)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    pool = [torch.randn(N, 12, device=dev, generator=gen) for _ in range(8)]
    env.reset()
    for i in range(args.warmup):
        env.step(pool[i % 8])

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    te = args.time_every
    reps = []
    for r in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if te:
                env.set_timing(i % te == 0, reset=False)  # sampled live per-kernel timing inside the timed region
            env.step(pool[i % 8])
        torch.cuda.synchronize(dev)
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            rank_el = el
            el = float(t.item())
        reps.append(el)
    kt = env.get_timing()
    env.set_timing(False)
    elapsed = sorted(reps)[len(reps) // 2]  # the median repeat (the only one at --repeats 1)
    ok = bool(torch.isfinite(env.root_states).all() and torch.isfinite(env.obs_buf).all())
    dist_info = {"backend": "none", "world_size": 1, "env_offsets": [env.env_offset]}
    if world > 1:
        # what the process group saw (a SCALE line shows whether RCCL had N ranks), each rank's shard and its own
        # elapsed time of the last repeat (the line's time is their max)
        shards = [None] * world
        torch.distributed.all_gather_object(shards, (int(env.env_offset), N, rank_el, bool(ok)))
        dist_info = {"backend": torch.distributed.get_backend(), "world_size": torch.distributed.get_world_size(),
                     "env_offsets": [s_[0] for s_ in shards], "envs_per_rank": [s_[1] for s_ in shards],
                     "rank_elapsed_s": [round(s_[2], 6) for s_ in shards]}
        ok = all(s_[3] for s_ in shards)
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    steps = args.steps
    value = N * world * steps / elapsed
    # live per-kernel HIP-event timing on the sampled steps
    fused = kt["k_post_a"]["launches"] == 0  # no split step inside the timed region: every launch is the whole step
    # at large N the history shift runs as its own launch ahead of the fused kernel (t1_shift_prelaunch)
    pre_shift = kt["k_shift"]["launches"] > 0
    per_kernel = {}
    cus = torch.cuda.get_device_properties(dev).multi_processor_count if torch.cuda.is_available() else 256
    FUSED_KERNEL = fused_kernel(N, cus, args.state_dtype == "fp16")
    for k in KERNELS + (["k_shift"] if pre_shift else []):
        ms = kt[k]["ms"] / max(1, kt[k]["launches"])
        if k == "k_shift":
            alg = shift_bytes * N
        elif fused and k == "k_dynamics":
            alg = (b_alg - (shift_bytes if pre_shift else 0)) * N
        else:
            alg = KERNEL_BYTES[k] * N
        name = FUSED_KERNEL if (fused and k == "k_dynamics") else k
        per_kernel[name] = {"avg_ms": round(ms, 5), "timed_launches": kt[k]["launches"], "alg_bytes_per_launch": alg,
                            "alg_GBs": round(alg / (ms * 1e-3) / 1e9, 1) if ms > 0 else None}
    step_span_ms = kt["step"]["ms"] / kt["step"]["launches"] if kt["step"]["launches"] else None
    # config 5 (k_dyn4, fp16 histories): the history shift runs as a concurrent launch (k_shift4c) on a second stream
    # beside the dynamics (T1ENV_D4_SHIFT, default on), so neither launch's own span is the step's: the pair is timed
    # as the step's fork-to-join span with the whole B_alg
    conc = pre_shift and FUSED_KERNEL == "k_dyn4" and os.environ.get("T1ENV_D4_SHIFT", "1") != "0"
    if conc and step_span_ms:
        per_kernel["k_dyn4 || k_shift4c"] = {
            "avg_ms": round(step_span_ms, 5), "timed_launches": kt["step"]["launches"], "alg_bytes_per_launch": b_alg * N,
            "alg_GBs": round(b_alg * N / (step_span_ms * 1e-3) / 1e9, 1), "note": "concurrent pair, fork-to-join span"}
        dom = "k_dyn4 || k_shift4c"
    else:
        dom = max(per_kernel, key=lambda k: per_kernel[k]["avg_ms"] * per_kernel[k]["timed_launches"])
    # roofline of the dominant kernel: its algorithmic bytes per launch (SURVEY.md §8(d) B_alg x envs when the launch
    # is the whole fused step) / its live HIP-event launch duration.  Without sampled events (--time-every 0) fall
    # back to the wall clock of the timed steps (env_steps_per_s x B_alg).
    dk = per_kernel[dom]
    if dk["alg_GBs"] is not None:
        achieved, basis = dk["alg_GBs"], f"{dom} alg bytes / live HIP-event launch duration"
    else:
        achieved, basis = value / world * b_alg / 1e9, "wall clock: env-steps/s x B_alg"
    traffic = None
    for path in ([args.traffic_json] if args.traffic_json else TRAFFIC_PROFILES):
        if not os.path.exists(path):
            continue
        try:
            tj = json.load(open(path))
            if tj.get("num_envs") == N and tj.get("mesh") == args.mesh and \
                    tj.get("state_dtype", "fp32") == args.state_dtype and bool(tj.get("push", False)) == bool(args.push):
                traffic = tj.get("hbm_bytes_per_step")
                break
        except Exception:
            traffic = None
    # the bound that binds: the fused kernel's dynamics waves are latency / VALU-issue bound.  VALU-issue
    # roofline: the VALU instructions (SQ counters, committed profile of the same workload) of a SIMD (k_dyn6: two role
    # waves, one instruction per 2 cycles) or of a dynamics wave (k_dyn5 / k_dyn4: one wave per SIMD, one per 4 cycles)
    # over the live launch duration.
    issue = None
    if fused and dom == FUSED_KERNEL and os.path.exists(args.sq_json) and dk["avg_ms"] > 0:
        try:
            sq = json.load(open(args.sq_json))
            if sq.get("envs") == N and args.mesh == "trimesh" and args.state_dtype == "fp32" and not args.push:
                ghz = sq["derived"].get("shader_clock_ghz", SHADER_GHZ)
                cyc = dk["avg_ms"] * 1e-3 * ghz * 1e9
                if sq.get("kernel") == "k_dyn6" == FUSED_KERNEL:
                    # two role waves per SIMD: the SIMD's VALU issue against one wave64 instruction per 2 cycles
                    insts, peak, unit = sq["derived"]["valu_insts_per_simd"], SIMD_VALU_PER_CYCLE, \
                        "VALU instr/cycle per SIMD (two role waves)"
                elif sq.get("kernel", "k_dyn5") == FUSED_KERNEL:
                    insts, peak, unit = sq["derived"]["valu_insts_per_dyn_wave"], LONE_WAVE_VALU_PER_CYCLE, \
                        "VALU instr/cycle per dynamics wave"
                else:
                    raise KeyError("the SQ profile is of another kernel")
                ach = insts / cyc
                issue = {"bound": "valu_issue", "unit": unit,
                         "achieved": round(ach, 4), "peak": peak,
                         "frac": round(ach / peak, 4),
                         "valu_insts": round(insts), "wave_cycles": round(cyc),
                         "shader_clock_ghz": round(ghz, 3),
                         "sq_profile_issue_frac": sq["derived"].get("simd_issue_frac",
                                                                    sq["derived"].get("dyn_wave_issue_frac")),
                         "wait_any_frac_all_waves": sq["derived"].get("wait_any_frac"),
                         "source": os.path.relpath(args.sq_json, REPO)}
        except Exception:
            issue = None
    # the bound: the roofline this kernel sits closest to.  HBM (achieved / peak below) unless the dynamics waves'
    # VALU-issue fraction is higher; when neither is near 1, SQ_WAIT_ANY says the rest is dependent latency
    hbm_frac = achieved / HBM_PEAK_GBS
    bound = "hbm"
    if issue is not None and issue["frac"] > hbm_frac:
        bound = "valu_issue"
    binding = {"hbm": f"HBM: {hbm_frac:.3f} of 8 TB/s"}
    if issue is not None:
        binding["valu_issue"] = f"{issue['unit']}: {issue['frac']:.3f} of {issue['peak']}"
        if max(hbm_frac, issue["frac"]) < 0.7:
            binding["note"] = ("neither roofline binds: dependent-latency / barrier waits of the core wave's chain "
                               f"(SQ_WAIT_ANY {issue['wait_any_frac_all_waves']:.2f} of wave cycles)"
                               if issue.get("wait_any_frac_all_waves") else "neither roofline binds: latency")
    line = {
        "metric": "env-steps/sec at 8192 envs, t1_dh_stand, 1/2/4/8 MI355X; obs/reward parity",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if args.state_dtype == "fp32" else "f32 compute, f16 obs/critic histories",
        "data": "synthetic",
        "config": {"workload": f"t1_dh_stand {N} envs/GPU, {args.mesh} curriculum terrain + full DR"
                               + (", pushes" if args.push else "") + ", random N(0,1) actions (policy excluded), "
                               f"10 substeps/step, {args.state_dtype} obs/critic histories",
                   "state_dtype": args.state_dtype,
                   "num_envs_per_gpu": N, "global_envs": N * world, "mesh": args.mesh, "parallelism": f"dp{world}"},
        "roofline": {"bound": bound, "kernel": dom, "basis": basis,
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "alg_bytes_per_step": b_alg * N, "alg_bytes_per_env_step": b_alg,
                     "wall_clock_GBs": round(value / world * b_alg / 1e9, 1),
                     "step_span_ms_timed": round(step_span_ms, 4) if step_span_ms else None,
                     "binding": binding,
                     "issue": issue,
                     "kernels": per_kernel},
        "finite": ok,
        "dist": dist_info,
        # the history buffers' device addresses (A/B records: step-time modes across processes vs buffer placement)
        "buffers": {k: hex(t.data_ptr()) for k, t in (("obs0", env._obs[0]), ("obs1", env._obs[1]),
                                                      ("priv0", env._priv[0]), ("priv1", env._priv[1]))}
                   if hasattr(env, "_priv") else None,
    }
    if len(reps) > 1:
        line["repeats"] = len(reps)
        line["repeat_values"] = [round(N * world * steps / e, 1) for e in reps]
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(env, args)
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
