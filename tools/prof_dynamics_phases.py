"""Dev probe: where k_dynamics spends its time, per substep phase (shader-clock deltas inside the kernel).

    python tools/prof_dynamics_phases.py --build      # here: builds _lib/libt1env_hip_prof.so (-DT1_PHASE_PROF)
    python tools/prof_dynamics_phases.py [--mesh trimesh] [--num-envs 8192]   # on the GPU box

Lane 0 of every dynamics wave accumulates clock64() deltas between the T1_PROF_MARK points of
t1env_dynamics.hip / t1_dynamics.h.  Reported per wave (0 = left leg, 1 = right leg) as the share of the
wave's cycles and as microseconds scaled to the measured kernel time.  The marks cost a few instructions
each, so the profiled kernel is slightly slower than the product one.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.path.join(REPO, "ti5_isaacgym_amd", "_lib", "libt1env_hip_prof.so")
BUCKETS = ["pd_torque+base_frame", "leg forward pass", "leg backward (no contact)", "leg contacts",
           "leg elimination", "base-box contacts", "LDS write + base block", "substep tail / loop",
           "barrier wait", "base solve + backsub + integrate", "prologue loads", "report (outputs)",
           "epilogue barrier", "post_a (fused)", "post_b (fused)", "handoff + zeroing + finalize"]
# k_dyn4 (4 waves): the same mark ids, with these meanings
BUCKETS4 = ["pd torques", "forward pass (+ pose publish)", "backward pass (no contact)", "shank + foot contacts",
            "contact fold-in + elimination", "base-box contacts",
            "base block", "substep loop / captures", "S1 wait (poses)", "base solve + backsub + integrate",
            "prologue loads", "S2 wait / report", "S3 wait / epilogue barrier", "post_a (fused)", "post_b (fused)",
            "handoff + zeroing + finalize"]
# finer marks inside the post-physics epilogue (t1env_postphys.h)
SUB = ["post_a: base quantities + feet euler", "post_a: callback (commands, push, ext force)",
       "post_a: termination + 24 rewards", "post_a: reward sum + episode sums",
       "post_b: reset_env (resetting lanes) + reload", "post_b: lag reads, phase, ref state",
       "post_b: privileged frame", "post_b: actor frame + noise"]
BUCKETS += SUB
BUCKETS4 += SUB
# the helper waves reuse ids 16-18 inside body_contact_np (they never run the epilogue)
HELPER_SUB = {16: "contacts: transforms + height queries (issue)", 17: "contacts: height-load latency",
              18: "contacts: contact math (points in contact)", 20: "helper kinematics (own + other leg)",
              21: "self-collision terms"}
NB = len(BUCKETS)
NW = 4
# k_dyn5 (t1env_dyn5.hip): per-role mark meanings (ids 13-15 epilogue and 16-23 sub-marks as above)
D5 = {  # bucket i = the time from the previous mark to mark i (t1env_dyn5.hip's T1_PROF_MARK ids)
    0: ["prologue", "S1 wait", "base frame, PD torques, base block, leg chain", "CRBA backward pass", "S2 wait",
        "LDS reads + fold-in", "elimination", "base system + solve + backsub + integrate", "log / captures / publish",
        "stores + R1 wait", "rigid report", "epilogue barrier"],
    1: ["prologue", "S1 wait", "state + base-box query issue", "RNEA bias + rhs", "base-box contact + halves",
        "publish + shift DMA retire", "S2 wait", "history shift slice", "-", "R1 wait", "base-box report",
        "epilogue barrier"],
    2: ["prologue + epilogue staging", "S1 wait", "state + kinematics", "foot / shank queries + shank contact",
        "foot contact (points 0-3)", "publish + shift DMA retire", "S2 wait", "history shift slice", "-", "R1 wait",
        "terrain report", "epilogue barrier"],
    3: ["prologue + epilogue staging", "S1 wait", "state + kinematics", "foot queries + self-contact terms",
        "foot contact (points 4-7)", "publish + shift DMA retire", "S2 wait", "history shift slice", "-", "R1 wait",
        "self-contact report", "epilogue barrier"],
}


# k_dyn6 (t1env_dyn6.hip, eight waves): mark meanings
D6_W0 = ["prologue", "S1 wait", "chain + CRBA", "S2 wait", "-", "LDS reads + fold-in", "elimination",
         "base system + solve + backsub + integrate + publish", "stores", "R1 wait", "rigid report", "RB wait",
         "epilogue barrier", "post_a (fused)", "post_a tail", "handoff + zeroing + finalize"]
D6_W4 = ["prologue + epilogue staging", "S1 wait", "capture, PD, base block, base box", "S2 wait", "-", "-", "-", "-",
         "-", "R1 wait", "capture stores + base-box report", "epilogue barrier"]
D6_R = ["-", "S1 wait", "role terms (pre-S2)", "S2 wait", "shift slice / prologue", "-", "-", "-",
        "shift store drain", "R1 wait", "report", "RB wait", "epilogue barrier", "-", "-", "epilogue (obs / state)"]
D6_ROLES = ["W0 core", "W1 RNEA", "W2 shank A", "W3 foot A", "W4 base", "W5 self", "W6 shank B", "W7 foot B"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true")
    p.add_argument("--mesh", default="trimesh")
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--split", action="store_true", help="time the split path (k_dynamics without epilogue)")
    p.add_argument("--no-self-collision", action="store_true", help="asset.self_collisions = 1 (A/B)")
    p.add_argument("--kernel", type=int, default=5, choices=[4, 5, 6], help="k_dyn5 (default), k_dyn6 or k_dyn4")
    p.add_argument("--lib", default=PROF_LIB, help="a profiling build (-DT1_PHASE_PROF), e.g. a what-if variant")
    a = p.parse_args()
    sys.path.insert(0, REPO)
    if a.build:
        from ti5_isaacgym_amd import build
        print(build.build(force=True, extra=["-DT1_PHASE_PROF"], out=PROF_LIB))
        return
    os.environ["T1ENV_LIB"] = a.lib
    os.environ["T1ENV_DYN_KERNEL"] = str(a.kernel)
    import torch
    from ti5_isaacgym_amd import make_t1_env
    def hook(cfg):
        if a.no_self_collision:
            cfg.asset.self_collisions = 1
    env = make_t1_env(num_envs=a.num_envs, mesh_type=a.mesh, seed=5, device="cuda:0", cfg_hook=hook)
    env.set_fused(not a.split)
    lib = ctypes.CDLL(a.lib)
    nw = 8 if a.kernel == 6 else NW
    buf = (ctypes.c_ulonglong * (nw * (24 if a.kernel == 6 else NB)))()
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.randn(a.num_envs, 12, device="cuda:0", generator=g) for _ in range(8)]
    for i in range(50):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    read = {5: lib.t1env_debug_phase_cycles5, 6: getattr(lib, "t1env_debug_phase_cycles6", None)}.get(
        a.kernel, lib.t1env_debug_phase_cycles)
    assert read(buf, 1) == 0
    env.set_timing(True)
    for i in range(a.steps):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    t = env.get_timing()
    env.set_timing(False)
    assert read(buf, 0) == 0
    kern_us = t["k_dynamics"]["ms"] / max(1, t["k_dynamics"]["launches"]) * 1e3
    waves = (a.num_envs + 63) // 64 if a.kernel == 4 else (a.num_envs + 31) // 32
    print(f"k_dynamics {kern_us:.1f} us/launch (events), {a.mesh}, {a.num_envs} envs, {a.steps} steps, "
          f"{'split' if a.split else 'fused'}")
    if a.kernel == 6:
        for w in range(8):
            cyc = [buf[w * 24 + i] / (waves * a.steps) for i in range(24)]
            tot = sum(cyc)
            names = D6_W0 if w == 0 else (D6_W4 if w == 4 else D6_R)
            print(f"wave {w} ({D6_ROLES[w]}): {tot:.0f} cycles/launch")
            for i, c in sorted(enumerate(cyc), key=lambda x: -x[1]):
                if c > 0:
                    nm = names[i] if i < len(names) else f"mark {i}"
                    print(f"   {nm:40s} {c:10.0f} cyc  {100 * c / tot:5.1f}%  ~{kern_us * c / tot:6.1f} us")
        return
    four = True
    names = BUCKETS4
    roles = ["left leg", "right leg", "left contact helper", "right contact helper"]
    if a.kernel == 5:
        roles = ["W0 core", "W1 bias", "W2 terrain", "W3 self"]
    for w in range(4):
        cyc = [buf[w * NB + i] / (waves * a.steps) for i in range(NB)]
        tot = sum(cyc)
        print(f"wave {w} ({roles[w]}): {tot:.0f} cycles/launch")
        if a.kernel == 5:
            wn = [D5[w][i] if i < len(D5[w]) else (HELPER_SUB.get(i, nm) if w >= 2 else nm)
                  for i, nm in enumerate(names)]
        else:
            wn = [HELPER_SUB.get(i, nm) if (four and w >= 2) else nm for i, nm in enumerate(names)]
        for name, c in sorted(zip(wn, cyc), key=lambda x: -x[1]):
            if c > 0:
                print(f"   {name:34s} {c:10.0f} cyc  {100 * c / tot:5.1f}%  ~{kern_us * c / tot:6.1f} us")


if __name__ == "__main__":
    main()
