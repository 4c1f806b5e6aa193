"""URDF -> collapsed articulation tables for the HIP dynamics (host-side, init time).

Replaces what Isaac Gym's ``gym.load_asset`` does for the reference (legged_robot.py:1276-1324 with
``collapse_fixed_joints=True``, legged_robot_config.py:103): every link reached from its parent through a
fixed joint is merged into that parent (mass summed, COM and inertia combined by the parallel-axis
theorem), leaving 13 bodies / 12 revolute DOF in Isaac Gym's depth-first order:
    0 base_link, 1-6 leg_l1..l6_link, 7-12 leg_r1..r6_link
(feet = the ``6_link`` bodies [6, 12], knees = ``4_link`` [4, 10]; legged_robot.py:1326-1335).

Collision geometry (contact candidates): the base box, the two shank boxes and the
two ankle-roll STL meshes (t1.urdf:42-51, 265-272, 390-398, 625-632, 750-758).  The mesh is replaced by
support points of its convex hull (sole corners, toe/heel edges), the box by its 8 corners.  Self-collision
volumes (``self_box``): the shank boxes themselves and the foot hulls' bounding boxes, in the link frame.
"""
import os
import struct
import xml.etree.ElementTree as ET

import numpy as np

BODY_NAMES = ["base_link"] + [f"leg_{s}{i}_link" for s in "lr" for i in range(1, 7)]
DOF_NAMES = [f"leg_{s}{i}_joint" for s in "lr" for i in range(1, 7)]
SELF_BODIES = [4, 6, 10, 12]   # leg_l4 (shank), leg_l6 (foot), leg_r4, leg_r6: the legs' collision bodies
FOOT_POINT_DIRS = [(1, 1, -1), (1, -1, -1), (-1, 1, -1), (-1, -1, -1),
                   (1, 0, -1), (-1, 0, -1), (1, 0, 0), (-1, 0, 0)]


def _rpy_to_R(rpy):
    r, p, y = rpy
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _vec(s, n=3):
    return np.array([float(x) for x in (s or " ".join(["0"] * n)).split()], dtype=np.float64)


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.zeros(3), np.eye(3)
    return _vec(o.get("xyz")), _rpy_to_R(_vec(o.get("rpy")))


def load_stl(path):
    b = open(path, "rb").read()
    if b[:5] == b"solid" and b"facet" in b[:300]:
        pts = [list(map(float, ln.split()[1:4])) for ln in b.decode().splitlines() if ln.strip().startswith("vertex")]
        return np.array(pts)
    n = struct.unpack("<I", b[80:84])[0]
    a = np.frombuffer(b[84:84 + n * 50], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    return a["v"].reshape(-1, 3).astype(np.float64)


def box_corners(size, xyz, R):
    s = np.asarray(size) / 2
    c = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * s
    return c @ R.T + xyz


class Articulation:
    """Collapsed articulation.  Arrays are float64; ``pack()`` flattens them for the C-ABI."""

    def __init__(self, urdf_path):
        self.urdf_path = urdf_path
        root = ET.parse(urdf_path).getroot()
        self.links = {l.get("name"): l for l in root.findall("link")}
        self.joints = root.findall("joint")
        by_parent = {}
        for j in self.joints:
            by_parent.setdefault(j.find("parent").get("link"), []).append(j)
        nb = len(BODY_NAMES)
        self.mass = np.zeros(nb)
        self.com = np.zeros((nb, 3))
        self.inertia = np.zeros((nb, 3, 3))   # about COM, body frame
        self.joint_offset = np.zeros((nb, 3))
        self.joint_axis = np.zeros((nb, 3))
        self.parent = np.full(nb, -1, dtype=np.int64)
        self.collisions = {b: [] for b in BODY_NAMES}
        jmap = {j.find("child").get("link"): j for j in self.joints}
        for b, name in enumerate(BODY_NAMES):
            if b > 0:
                j = jmap[name]
                assert j.get("type") == "revolute", name
                xyz, R = _origin(j)
                assert np.allclose(R, np.eye(3)), "leg joints carry no rpy in t1.urdf"
                self.joint_offset[b] = xyz
                self.joint_axis[b] = _vec(j.find("axis").get("xyz"))
                self.parent[b] = BODY_NAMES.index(j.find("parent").get("link"))
            # merge this link and every fixed descendant into body b
            parts = [(name, np.zeros(3), np.eye(3))]
            stack = [(name, np.zeros(3), np.eye(3))]
            while stack:
                ln, p, R = stack.pop()
                for j in by_parent.get(ln, []):
                    if j.get("type") != "fixed":
                        continue
                    xyz, Rj = _origin(j)
                    child = j.find("child").get("link")
                    item = (child, p + R @ xyz, R @ Rj)
                    parts.append(item)
                    stack.append(item)
            m_tot, mc = 0.0, np.zeros(3)
            pieces = []
            for ln, p, R in parts:
                inert = self.links[ln].find("inertial")
                m = float(inert.find("mass").get("value"))
                cxyz, cR = _origin(inert)
                I = inert.find("inertia")
                Il = np.array([[float(I.get("ixx")), float(I.get("ixy")), float(I.get("ixz"))],
                               [float(I.get("ixy")), float(I.get("iyy")), float(I.get("iyz"))],
                               [float(I.get("ixz")), float(I.get("iyz")), float(I.get("izz"))]])
                Rb = R @ cR
                c = p + R @ cxyz
                pieces.append((m, c, Rb @ Il @ Rb.T))
                m_tot += m
                mc += m * c
                for col in self.links[ln].findall("collision"):
                    cx, cR2 = _origin(col)
                    g = col.find("geometry")[0]
                    self.collisions[name].append((g.tag, g.attrib, p + R @ cx, R @ cR2))
            c = mc / m_tot
            Ic = np.zeros((3, 3))
            for m, ci, Ii in pieces:
                d = ci - c
                Ic += Ii + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
            self.mass[b], self.com[b], self.inertia[b] = m_tot, c, Ic
        self.limits = np.zeros((12, 4))   # lower, upper, effort, velocity
        for i, n in enumerate(DOF_NAMES):
            lim = [j for j in self.joints if j.get("name") == n][0].find("limit")
            self.limits[i] = [float(lim.get("lower")), float(lim.get("upper")), float(lim.get("effort")),
                              float(lim.get("velocity"))]
        self._contact_points()

    def _contact_points(self):
        mesh_dir = os.path.dirname(self.urdf_path)
        pts, bodies = [], []
        self.self_box = {}   # body -> [center (3), half extents (3)] in the link frame (self-collision volumes)
        for b, name in enumerate(BODY_NAMES):
            for tag, attr, xyz, R in self.collisions[name]:
                if tag == "box":
                    c = box_corners(_vec(attr["size"]), xyz, R)
                    if not np.allclose(R, np.eye(3)) and b != 0:
                        raise ValueError("rotated leg collision boxes are not supported")
                    self.self_box[b] = list(xyz) + list(_vec(attr["size"]) / 2)
                elif tag == "mesh":
                    v = load_stl(os.path.normpath(os.path.join(mesh_dir, attr["filename"])))
                    v = v @ R.T + xyz
                    c = np.array([v[np.argmax(v @ np.asarray(d, float))] for d in FOOT_POINT_DIRS])
                    # the hull's axis-aligned bounding box in the link frame stands in for the hull as a self-collision
                    # volume (PhysX collides the convex hull itself)
                    lo, hi = v.min(0), v.max(0)
                    self.self_box[b] = list((lo + hi) / 2) + list((hi - lo) / 2)
                else:
                    raise ValueError(f"unsupported collision geometry {tag}")
                pts.extend(c)
                bodies.extend([b] * len(c))
        order = np.argsort(bodies, kind="stable")
        self.contact_body = np.asarray(bodies)[order]
        self.contact_point = np.asarray(pts)[order]
        self.contact_start = np.zeros(len(BODY_NAMES), np.int32)
        self.contact_count = np.zeros(len(BODY_NAMES), np.int32)
        for b in range(len(BODY_NAMES)):
            idx = np.nonzero(self.contact_body == b)[0]
            self.contact_count[b] = len(idx)
            self.contact_start[b] = idx[0] if len(idx) else 0


RESOURCE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "resources", "t1_model.json")


def compile_model(urdf_path):
    """Articulation tables as a JSON-able dict (what t1env_model needs besides the solver constants)."""
    a = Articulation(urdf_path)
    return {
        "source": os.path.basename(urdf_path),
        "body_names": BODY_NAMES, "dof_names": DOF_NAMES,
        "parent": a.parent.tolist(), "mass": a.mass.tolist(), "com": a.com.tolist(),
        "inertia": [[I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]] for I in a.inertia],
        "joint_offset": a.joint_offset.tolist(), "joint_axis": a.joint_axis.tolist(),
        "limits": a.limits.tolist(),  # lower, upper, effort, velocity
        "contact_body": a.contact_body.tolist(), "contact_point": a.contact_point.tolist(),
        "contact_start": a.contact_start.tolist(), "contact_count": a.contact_count.tolist(),
        # self-collision boxes of left shank, left foot, right shank, right foot (center, half extents; link frame)
        "self_box": [[float(x) for x in a.self_box[b]] for b in SELF_BODIES],
    }


def self_capsules(tab):
    """The self-collision capsules of left shank, left foot, right shank, right foot, from the model's boxes
    (``self_box``): along the box's longest axis, radius the smaller of its two cross-section half extents (the shank's
    0.05 m square section; the foot's lateral half width, the direction the feet meet each other in), segment ends
    inset by the radius so the capsule spans the box's length.  Rows: a (3), b (3), radius, link frame."""
    out = []
    for box in tab["self_box"]:
        c, h = np.asarray(box[:3], float), np.asarray(box[3:], float)
        ax = int(np.argmax(h))
        r = float(min(h[k] for k in range(3) if k != ax))
        e = np.zeros(3)
        e[ax] = max(h[ax] - r, 1e-3)
        out.append([float(x) for x in np.concatenate([c - e, c + e, [r]])])
    return out


def load_model(urdf_path=None):
    """Compiled tables: from a URDF when given (and present), else the committed t1_model.json."""
    import json
    if urdf_path and os.path.exists(urdf_path):
        return compile_model(urdf_path)
    with open(RESOURCE) as f:
        return json.load(f)


if __name__ == "__main__":
    import json
    import sys
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/resources/robots/t1/urdf/t1.urdf"
    os.makedirs(os.path.dirname(RESOURCE), exist_ok=True)
    with open(RESOURCE, "w") as f:
        json.dump(compile_model(src), f, indent=1)
    print("wrote", RESOURCE)
