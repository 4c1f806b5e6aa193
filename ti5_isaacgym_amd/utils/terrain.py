"""Curriculum height-field terrain (host side, built once at env creation).

Follows humanoid/utils/terrain.py:9-191 (sub-terrain grid, difficulty per row, type per column,
env origins on the central platform) and restates the Isaac Gym Preview 4 ``terrain_utils`` helpers it
calls (random_uniform_terrain, pyramid_sloped_terrain, pyramid_stairs_terrain, discrete_obstacles_terrain,
wave_terrain) -- third-party code absent from the image, so the helper arithmetic is *parity unpinned*;
the layout/origins/curriculum logic is pinned by tests/test_terrain.py against the golden fixture.

Random draws use numpy's global generator in the reference's call order (seeded by ``set_seed``), so the
same seed reproduces the reference's height field.  The triangle mesh the reference builds from the
height field (``convert_heightfield_to_trimesh``) is not materialised: the HIP contact query samples the
height field with the same two-triangles-per-cell split (t1_dynamics.h: terrain_height).
"""
import numpy as np
from scipy.interpolate import RegularGridInterpolator


class SubTerrain:
    def __init__(self, width, length, vertical_scale, horizontal_scale):
        self.width, self.length = width, length
        self.vertical_scale, self.horizontal_scale = vertical_scale, horizontal_scale
        self.height_field_raw = np.zeros((width, length), dtype=np.int16)


def random_uniform_terrain(t, min_height, max_height, step=1.0, downsampled_scale=None):
    if downsampled_scale is None:
        downsampled_scale = t.horizontal_scale
    lo, hi, st = int(min_height / t.vertical_scale), int(max_height / t.vertical_scale), int(step / t.vertical_scale)
    heights = np.arange(lo, hi + st, st)
    coarse = np.random.choice(heights, (int(t.width * t.horizontal_scale / downsampled_scale),
                                        int(t.length * t.horizontal_scale / downsampled_scale)))
    gx = np.linspace(0, t.width * t.horizontal_scale, coarse.shape[0])
    gy = np.linspace(0, t.length * t.horizontal_scale, coarse.shape[1])
    interp = RegularGridInterpolator((gx, gy), coarse.astype(np.float64), method="linear")
    fx = np.linspace(0, t.width * t.horizontal_scale, t.width)
    fy = np.linspace(0, t.length * t.horizontal_scale, t.length)
    X, Y = np.meshgrid(fx, fy, indexing="ij")
    up = np.rint(interp(np.stack([X.ravel(), Y.ravel()], 1)).reshape(t.width, t.length))
    t.height_field_raw += up.astype(np.int16)


def pyramid_sloped_terrain(t, slope=1.0, platform_size=1.0):
    cx, cy = int(t.width / 2), int(t.length / 2)
    xx = ((cx - np.abs(cx - np.arange(t.width))) / cx).reshape(t.width, 1)
    yy = ((cy - np.abs(cy - np.arange(t.length))) / cy).reshape(1, t.length)
    peak = int(slope * (t.horizontal_scale / t.vertical_scale) * (t.width / 2))
    t.height_field_raw += (peak * xx * yy).astype(t.height_field_raw.dtype)
    p = int(platform_size / t.horizontal_scale / 2)
    x1, y1 = t.width // 2 - p, t.length // 2 - p
    edge = t.height_field_raw[x1, y1]
    t.height_field_raw = np.clip(t.height_field_raw, min(edge, 0), max(edge, 0))


def pyramid_stairs_terrain(t, step_width, step_height, platform_size=1.0):
    w, h, p = int(step_width / t.horizontal_scale), int(step_height / t.vertical_scale), int(platform_size / t.horizontal_scale)
    level, x0, x1, y0, y1 = 0, 0, t.width, 0, t.length
    while (x1 - x0) > p and (y1 - y0) > p:
        x0, x1, y0, y1, level = x0 + w, x1 - w, y0 + w, y1 - w, level + h
        t.height_field_raw[x0:x1, y0:y1] = level


def discrete_obstacles_terrain(t, max_height, min_size, max_size, num_rects, platform_size=1.0):
    mh = int(max_height / t.vertical_scale)
    lo, hi = int(min_size / t.horizontal_scale), int(max_size / t.horizontal_scale)
    p = int(platform_size / t.horizontal_scale)
    heights = [-mh, -mh // 2, mh // 2, mh]
    widths, lengths = range(lo, hi, 4), range(lo, hi, 4)
    for _ in range(num_rects):
        w, l = np.random.choice(widths), np.random.choice(lengths)
        sx, sy = np.random.choice(range(0, t.width - w, 4)), np.random.choice(range(0, t.length - l, 4))
        t.height_field_raw[sx:sx + w, sy:sy + l] = np.random.choice(heights)
    x1, x2 = (t.width - p) // 2, (t.width + p) // 2
    y1, y2 = (t.length - p) // 2, (t.length + p) // 2
    t.height_field_raw[x1:x2, y1:y2] = 0


def wave_terrain(t, num_waves=1, amplitude=1.0):
    amp = int(0.5 * amplitude / t.vertical_scale)
    if num_waves > 0:
        div = t.length / (num_waves * np.pi * 2)
        x, y = np.arange(0, t.width), np.arange(0, t.length)
        xx, yy = np.meshgrid(x, y, sparse=True)
        t.height_field_raw += (amp * np.cos(yy.reshape(1, t.length) / div)
                               + amp * np.sin(xx.reshape(t.width, 1) / div)).astype(t.height_field_raw.dtype)


def gap_terrain(t, gap_size, platform_size=1.0):
    g, p = int(gap_size / t.horizontal_scale), int(platform_size / t.horizontal_scale)
    cx, cy = t.length // 2, t.width // 2
    x1, y1 = (t.length - p) // 2, (t.width - p) // 2
    x2, y2 = x1 + g, y1 + g
    t.height_field_raw[cx - x2:cx + x2, cy - y2:cy + y2] = -1000
    t.height_field_raw[cx - x1:cx + x1, cy - y1:cy + y1] = 0


def pit_terrain(t, depth, platform_size=1.0):
    d, p = int(depth / t.vertical_scale), int(platform_size / t.horizontal_scale / 2)
    t.height_field_raw[t.length // 2 - p:t.length // 2 + p, t.width // 2 - p:t.width // 2 + p] = -d


class Terrain:
    """Height field + per-(level, type) env origins (reference terrain.py:9-50, 173-191)."""

    def __init__(self, cfg, num_robots):
        self.cfg, self.type = cfg, cfg.mesh_type
        if self.type in ("none", "plane"):
            return
        self.env_length, self.env_width = cfg.terrain_length, cfg.terrain_width
        props = np.array(cfg.terrain_proportions, dtype=np.float64)
        props = props / props.sum()
        self.proportions = [float(np.sum(props[:i + 1])) for i in range(len(props))]
        self.num_rows, self.num_cols = cfg.num_rows, cfg.num_cols
        self.env_origins = np.zeros((cfg.num_rows, cfg.num_cols, 3))
        self.max_difficulty = (cfg.num_rows - 1) / cfg.num_rows
        self.hs, self.vs = cfg.horizontal_scale, cfg.vertical_scale
        self.width_px = int(self.env_width / self.hs)
        self.length_px = int(self.env_length / self.hs)
        self.border = int(cfg.border_size / self.hs)
        self.tot_cols = int(cfg.num_cols * self.width_px) + 2 * self.border
        self.tot_rows = int(cfg.num_rows * self.length_px) + 2 * self.border
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        self.terrain_type = np.zeros((cfg.num_rows, cfg.num_cols))
        self.idx = 0
        if cfg.curriculum:
            for j in range(cfg.num_cols):
                for i in range(cfg.num_rows):
                    self._add(self.make_terrain(j / cfg.num_cols + 0.001, i / cfg.num_rows), i, j)
        else:
            for k in range(cfg.num_rows * cfg.num_cols):
                i, j = np.unravel_index(k, (cfg.num_rows, cfg.num_cols))
                choice = np.random.uniform(0, 1)
                difficulty = np.random.choice([0.5, 0.75, 0.9])
                self._add(self.make_terrain(choice, difficulty), i, j)
        self.heightsamples = self.height_field_raw

    def _lerp(self, rng, difficulty):
        return rng[0] + difficulty * (rng[1] - rng[0]) / self.max_difficulty

    def make_terrain(self, choice, difficulty):
        c = self.cfg
        t = SubTerrain(self.width_px, self.width_px, c.vertical_scale, c.horizontal_scale)
        rf_lo = -c.rough_flat_range[0] - difficulty * (c.rough_flat_range[1] - c.rough_flat_range[0]) / self.max_difficulty
        rf_hi = self._lerp(c.rough_flat_range, difficulty)
        slope = self._lerp(c.slope_range, difficulty)
        rs_lo = -c.rough_slope_range[0] - difficulty * (c.rough_slope_range[1] - c.rough_slope_range[0]) / self.max_difficulty
        rs_hi = self._lerp(c.rough_slope_range, difficulty)
        stair_w = self._lerp(c.stair_width_range, difficulty)
        stair_h = self._lerp(c.stair_height_range, difficulty)
        disc_h = self._lerp(c.discrete_height_range, difficulty)
        P = self.proportions
        if choice < P[0]:
            self.idx = 1
        elif choice < P[1]:
            self.idx = 2
            random_uniform_terrain(t, rf_lo, rf_hi, step=0.005, downsampled_scale=0.2)
        elif choice < P[3]:
            self.idx = 4
            if choice < P[2]:
                self.idx, slope = 3, -slope
            pyramid_sloped_terrain(t, slope=slope, platform_size=c.platform)
            random_uniform_terrain(t, rs_lo, rs_hi, step=0.005, downsampled_scale=0.2)
        elif choice < P[5]:
            self.idx = 6
            if choice < P[4]:
                self.idx, slope = 5, -slope
            pyramid_sloped_terrain(t, slope=slope, platform_size=c.platform)
        elif choice < P[7]:
            self.idx = 8
            if choice < P[6]:
                self.idx, stair_h = 7, -stair_h
            pyramid_stairs_terrain(t, step_width=stair_w, step_height=stair_h, platform_size=c.platform)
        elif choice < P[8]:
            self.idx = 9
            discrete_obstacles_terrain(t, disc_h, 1.0, 2.0, 20, platform_size=c.platform)
        elif choice < P[9]:
            self.idx = 10
            wave_terrain(t, num_waves=3, amplitude=0.2 + 0.333 * difficulty)
        elif len(P) > 10 and choice < P[10]:
            self.idx = 11
            gap_terrain(t, gap_size=1.0 * difficulty, platform_size=c.platform)
        else:
            self.idx = 12
            pit_terrain(t, depth=1.0 * difficulty, platform_size=c.platform)
        return t

    def _add(self, t, row, col):
        x0, x1 = self.border + row * self.length_px, self.border + (row + 1) * self.length_px
        y0, y1 = self.border + col * self.width_px, self.border + (col + 1) * self.width_px
        self.height_field_raw[x0:x1, y0:y1] = t.height_field_raw
        ox, oy = (row + 0.5) * self.env_length, (col + 0.5) * self.env_width
        a1, a2 = int((self.env_length / 2.0 - 1) / t.horizontal_scale), int((self.env_length / 2.0 + 1) / t.horizontal_scale)
        b1, b2 = int((self.env_width / 2.0 - 1) / t.horizontal_scale), int((self.env_width / 2.0 + 1) / t.horizontal_scale)
        oz = np.max(t.height_field_raw[a1:a2, b1:b2]) * t.vertical_scale
        self.env_origins[row, col] = [ox, oy, oz]
        self.terrain_type[row, col] = self.idx
