"""CPU baseline env (TEST INFRASTRUCTURE / bench.py cpu_baseline leg only).

The reference's own CPU path (Isaac Gym PhysX CPU + torch CPU) cannot run here or on the GPU box, so the
CPU baseline is the build's restatement: the numpy oracle for PD + post-physics (oracle/t1_oracle.py)
plus the dynamics header compiled for the host with OpenMP (oracle/dyn_cpu.cpp), fp32.
"""
import ctypes as C
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import build_cpu
from .t1_oracle import T1Oracle


class CpuT1Env:
    def __init__(self, model, num_envs, seed=5, mesh_type="plane", terrain=None, fp64=False, env_offset=0,
                 reduce_fn=None, omp_threads=None):
        self.lib = C.CDLL(build_cpu.build())
        self.model = model
        self.omp_threads = omp_threads
        self.o = T1Oracle(num_envs, seed=seed, mesh_type=mesh_type, terrain=terrain, env_offset=env_offset,
                          reduce_fn=reduce_fn)
        self.fp64 = int(fp64)
        self.N = num_envs
        if terrain is not None and mesh_type in ("heightfield", "trimesh"):
            self.hf = np.ascontiguousarray(terrain["height_samples"], np.int16)
            self.tparams = (self.hf.shape[0], self.hf.shape[1], terrain.get("horizontal_scale", 0.1),
                            terrain.get("vertical_scale", 0.005), terrain.get("border_size", 25.0), 2)
        else:
            self.hf = np.zeros((2, 2), np.int16)
            self.tparams = (2, 2, 0.1, 0.005, 0.0, 0)
        self.rigid = np.zeros((num_envs, 13, 13), np.float32)
        self.vimp = np.zeros((num_envs, 6), np.float32)   # the contact bodies' restitution episodes (t1_dynamics.h)
        self.contact = np.zeros((num_envs, 13, 3), np.float32)

    def threads(self):
        return int(self.lib.t1dyn_num_threads())

    def _physics(self, g, torques, o):
        fp = C.POINTER(C.c_float)
        f = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
        root, dof = f(o.root.copy()), f(o.dof.reshape(self.N, 24).copy())
        args = [f(torques), f(o.body_mass), f(o.link_mass_scale), f(o.com_disp), f(o.armature), f(o.friction),
                f(o.restitution)]
        ext = f(o.applied_force[:, 0, :]) if o.force_pending else None
        rows, cols, hs, vs, border, mesh = self.tparams
        if self.omp_threads:
            self.lib.t1dyn_set_num_threads(int(self.omp_threads))   # this calling thread's OpenMP team size
        rc = self.lib.t1dyn_substeps(
            C.byref(self.model), self.N, self.fp64, root.ctypes.data_as(fp), dof.ctypes.data_as(fp),
            *[a.ctypes.data_as(fp) for a in args], self.vimp.ctypes.data_as(fp),
            ext.ctypes.data_as(fp) if ext is not None else None,
            C.c_float(0.001), 1, self.hf.ctypes.data_as(C.POINTER(C.c_int16)), rows, cols, C.c_float(hs),
            C.c_float(vs), C.c_float(border), mesh, self.rigid.ctypes.data_as(fp), self.contact.ctypes.data_as(fp))
        assert rc == 0
        return root, dof.reshape(self.N, 12, 2), self.rigid.copy(), self.contact.copy()

    def reset(self):
        return self.o.reset(self._physics)

    def step(self, actions):
        return self.o.step(np.asarray(actions, np.float32), self._physics)


class ShardedCpuT1Env:
    """The CPU baseline on every host core: S shards of the env (global ids [s N/S, (s+1) N/S), like the multi-GPU
    shards, so every draw and terrain type is the unsharded run's), each stepped by its own Python thread -- the numpy
    post-physics releases the GIL in its array kernels -- with its physics on cores / S OpenMP threads.  The command
    curriculum's global mean is reduced over the shards (the oracle's reduce_fn)."""

    def __init__(self, model, num_envs, cores, shards=None, seed=5, mesh_type="plane", terrain=None):
        S = max(1, min(shards or min(cores, 16), num_envs))
        bounds = [num_envs * s // S for s in range(S + 1)]
        self.bounds = bounds
        self._bar = threading.Barrier(S)
        self._acc = [0.0, 0]
        self._lock = threading.Lock()
        per = max(1, cores // S)
        self.cores = per * S
        t = None
        if terrain is not None:
            t = dict(terrain, num_envs_total=num_envs)
        self.shards = [CpuT1Env(model, bounds[s + 1] - bounds[s], seed=seed, mesh_type=mesh_type, terrain=t,
                                env_offset=bounds[s], reduce_fn=self._reduce if S > 1 else None, omp_threads=per)
                       for s in range(S)]
        self.pool = ThreadPoolExecutor(S)

    BARRIER_TIMEOUT_S = 600.0   # a stuck shard cannot hang the CPU baseline

    def _reduce(self, s, c):
        if self._bar.wait(self.BARRIER_TIMEOUT_S) == 0:
            self._acc = [0.0, 0]
        self._bar.wait(self.BARRIER_TIMEOUT_S)
        with self._lock:
            self._acc[0] += s
            self._acc[1] += c
        self._bar.wait(self.BARRIER_TIMEOUT_S)
        return self._acc[0], self._acc[1]

    def threads(self):
        return self.cores

    def reset(self):
        list(self.pool.map(lambda e: e.reset(), self.shards))

    def step(self, actions):
        b = self.bounds

        def one(i):
            try:
                return self.shards[i].step(actions[b[i]:b[i + 1]])
            except BaseException:
                # a shard that fails before or inside the curriculum reduction breaks the barrier, so the other shards
                # raise BrokenBarrierError instead of waiting forever; the first error propagates
                self._bar.abort()
                raise
        list(self.pool.map(one, range(len(self.shards))))
