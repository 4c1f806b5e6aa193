"""Stand-in for isaacgym.gymapi: value types + ``acquire_gym`` returning the harness FakeGym."""
import numpy as np

SIM_PHYSX = 1
SIM_FLEX = 0
ENV_SPACE = 1
LOCAL_SPACE = 0
KEY_ESCAPE = 0
KEY_V = 1
UP_AXIS_Z = 1
DOF_MODE_EFFORT = 3


class Vec3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __add__(self, o):
        return Vec3(self.x + o.x, self.y + o.y, self.z + o.z)

    def __repr__(self):
        return f"Vec3({self.x}, {self.y}, {self.z})"


class Quat:
    def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
        self.x, self.y, self.z, self.w = x, y, z, w


class Transform:
    def __init__(self, p=None, r=None):
        self.p = p if p is not None else Vec3()
        self.r = r if r is not None else Quat()


class _Bag:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class SimParams:
    def __init__(self):
        self.dt = 0.01
        self.substeps = 1
        self.up_axis = UP_AXIS_Z
        self.gravity = Vec3(0, 0, -9.81)
        self.use_gpu_pipeline = False
        self.physx = _Bag(use_gpu=False, num_subscenes=0, num_threads=0, solver_type=1,
                          num_position_iterations=4, num_velocity_iterations=0, contact_offset=0.01,
                          rest_offset=0.0, bounce_threshold_velocity=0.5, max_depenetration_velocity=1.0,
                          max_gpu_contact_pairs=2 ** 23, default_buffer_size_multiplier=5,
                          contact_collection=2)


class PlaneParams:
    def __init__(self):
        self.normal = Vec3(0, 0, 1)
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0


class HeightFieldParams(_Bag):
    def __init__(self):
        super().__init__(transform=Transform())


class TriangleMeshParams(_Bag):
    def __init__(self):
        super().__init__(transform=Transform())


class AssetOptions(_Bag):
    pass


class CameraProperties(_Bag):
    pass


def acquire_gym():
    import fake_gym
    return fake_gym.FakeGym.instance()
