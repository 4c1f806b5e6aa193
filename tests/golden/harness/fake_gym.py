"""TEST-ONLY FakeGym: answers the gym.* calls the reference env makes, with physics replaced by injection.

``simulate()`` does no physics: it asks the installed provider for the next (root, dof, rigid, contact)
state and writes it into the tensors the reference wrapped via gymtorch (zero-copy in Isaac Gym too).
Everything the reference *sends* to the simulator (torques, external forces, DOF properties) is recorded
so the golden vectors can pin our PD / ext-force / DR paths.
"""
import copy
import os
import xml.etree.ElementTree as ET

import numpy as np
import torch

from isaacgym import gymapi

REF_ROOT = os.environ.get("T1_REFERENCE_ROOT", "/root/reference")
URDF = os.path.join(REF_ROOT, "resources/robots/t1/urdf/t1.urdf")


def _robot_tables():
    """Body/DOF names, collapsed masses and DOF limits straight from the URDF (Isaac Gym DFS order)."""
    root = ET.parse(URDF).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    body_names = ["base_link"] + [f"leg_{s}{i}_link" for s in "lr" for i in range(1, 7)]
    dof_names = [f"leg_{s}{i}_joint" for s in "lr" for i in range(1, 7)]
    masses = []
    for b in body_names:
        masses.append(float(links[b].find("inertial").find("mass").get("value")))
    # collapse_fixed_joints: every link reached from base_link through fixed joints merges into it
    fixed_children = {}
    for j in joints:
        if j.get("type") == "fixed":
            fixed_children.setdefault(j.find("parent").get("link"), []).append(j.find("child").get("link"))
    stack, extra = ["base_link"], 0.0
    while stack:
        for c in fixed_children.get(stack.pop(), []):
            extra += float(links[c].find("inertial").find("mass").get("value"))
            stack.append(c)
    masses[0] += extra
    jmap = {j.get("name"): j for j in joints}
    dt = np.dtype([("hasLimits", bool), ("lower", np.float32), ("upper", np.float32), ("driveMode", np.int32),
                   ("velocity", np.float32), ("effort", np.float32), ("stiffness", np.float32),
                   ("damping", np.float32), ("friction", np.float32), ("armature", np.float32)])
    props = np.zeros(len(dof_names), dtype=dt)
    for i, n in enumerate(dof_names):
        lim = jmap[n].find("limit")
        props[i] = (True, float(lim.get("lower")), float(lim.get("upper")), 3, float(lim.get("velocity")),
                    float(lim.get("effort")), 0.0, 0.0, 0.0, 0.0)
    return body_names, dof_names, masses, props


class _Obj:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class FakeGym:
    _inst = None

    @classmethod
    def instance(cls):
        if cls._inst is None:
            cls._inst = FakeGym()
        return cls._inst

    @classmethod
    def reset_instance(cls):
        cls._inst = None

    def __init__(self):
        self.body_names, self.dof_names, self.masses, self.dof_props = _robot_tables()
        self.num_envs = 0
        self.provider = None
        self.substep = 0
        self.torque_log = []
        self.force_log = []
        self.dof_prop_log = {}
        self.tensors = None

    # ---- creation -----------------------------------------------------------------------------
    def create_sim(self, *a, **k):
        return "sim"

    def add_ground(self, sim, params):
        self.ground = params

    def add_heightfield(self, sim, hf, params):
        self.heightfield = (hf, params)

    def add_triangle_mesh(self, sim, v, t, params):
        self.trimesh = (v, t, params)

    def load_asset(self, sim, root, file, opts):
        return "asset"

    def get_asset_dof_count(self, a):
        return len(self.dof_names)

    def get_asset_rigid_body_count(self, a):
        return len(self.body_names)

    def get_asset_dof_properties(self, a):
        return self.dof_props.copy()

    def get_asset_rigid_shape_properties(self, a):
        return [_Obj(friction=1.0, restitution=0.0) for _ in range(5)]

    def set_asset_rigid_shape_properties(self, a, props):
        pass

    def get_asset_rigid_body_names(self, a):
        return list(self.body_names)

    def get_asset_dof_names(self, a):
        return list(self.dof_names)

    def create_env(self, sim, lo, hi, per_row):
        self.num_envs += 1
        return self.num_envs - 1

    def create_actor(self, env, asset, pose, name, group, filt, seg):
        self.start_poses = getattr(self, "start_poses", {})
        self.start_poses[env] = (pose.p.x, pose.p.y, pose.p.z)
        return 0

    def set_actor_dof_properties(self, env, actor, props):
        self.dof_prop_log[env] = np.array(props["armature"], dtype=np.float32).copy()

    def get_actor_dof_properties(self, env, actor):
        return self.dof_props.copy()

    def get_actor_rigid_body_properties(self, env, actor):
        return [_Obj(mass=m, com=gymapi.Vec3(), inertia=_Obj(x=gymapi.Vec3(), y=gymapi.Vec3(), z=gymapi.Vec3()))
                for m in self.masses]

    def set_actor_rigid_body_properties(self, env, actor, props, recomputeInertia=False):
        pass

    def find_actor_rigid_body_handle(self, env, actor, name):
        return self.body_names.index(name)

    def prepare_sim(self, sim):
        n, nb, nd = self.num_envs, len(self.body_names), len(self.dof_names)
        self.tensors = dict(root=torch.zeros(n, 13), dof=torch.zeros(n * nd, 2),
                            contact=torch.zeros(n * nb, 3), rigid=torch.zeros(n * nb, 13))
        self.tensors["root"][:, 6] = 1.0
        # like Isaac Gym after prepare_sim: root states hold the actors' start poses
        for e, p in getattr(self, "start_poses", {}).items():
            self.tensors["root"][e, 0:3] = torch.tensor(p)

    def create_camera_sensor(self, env, props):
        return 0

    # ---- tensor API ---------------------------------------------------------------------------
    def acquire_actor_root_state_tensor(self, sim):
        return self.tensors["root"]

    def acquire_dof_state_tensor(self, sim):
        return self.tensors["dof"]

    def acquire_net_contact_force_tensor(self, sim):
        return self.tensors["contact"]

    def acquire_rigid_body_state_tensor(self, sim):
        return self.tensors["rigid"]

    def refresh_dof_state_tensor(self, sim):
        pass

    def refresh_actor_root_state_tensor(self, sim):
        pass

    def refresh_net_contact_force_tensor(self, sim):
        pass

    def refresh_rigid_body_state_tensor(self, sim):
        pass

    def set_dof_actuation_force_tensor(self, sim, t):
        self.torque_log.append(t.clone())

    def apply_rigid_body_force_tensors(self, sim, forces, torques, space):
        self.force_log.append((forces.clone(), torques.clone()))

    def set_dof_state_tensor_indexed(self, sim, state, ids, n):
        pass

    def set_actor_root_state_tensor_indexed(self, sim, state, ids, n):
        pass

    def set_actor_root_state_tensor(self, sim, state):
        pass

    def simulate(self, sim):
        if self.provider is not None:
            self.provider(self.tensors, self.substep)
        self.substep += 1

    def fetch_results(self, sim, wait):
        pass
