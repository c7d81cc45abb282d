"""Training data for the online trainer (BASELINE config 5).

* `load_nerf_synthetic` reads a NeRF-synthetic scene (transforms.json + 8-bit PNGs, e.g. the lego
  set the reference ships under data/nerf/lego) the way ngp's loader does (nerf_loader.cu:
  focal from fl_x / camera_angle_x, principal point cx/w or 0.5, scale 0.33, offset 0.5, and
  `nerf_matrix_to_ngp`, nerf_loader.h:101-120).
* `render_views` makes a synthetic training set by rendering a model with the instant-NGP
  render path (ground truth for convergence and parity tests without any dataset).
"""
import ctypes
import json
import math
import os

import numpy as np

from . import _lib

NERF_SCALE = 0.33   # nerf_loader.cu: result.scale = NERF_SCALE


def read_png(path):
    """8-bit PNG -> [h, w, 4] uint8 (libsng_hip's host decoder)."""
    lib = _lib.load()
    w, h = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(lib.sng_image_load_png(str(path).encode(), None, 0, ctypes.byref(w), ctypes.byref(h)))
    out = np.zeros((h.value, w.value, 4), np.uint8)
    _lib.check(lib.sng_image_load_png(str(path).encode(), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.nbytes, ctypes.byref(w),
                                      ctypes.byref(h)))
    return out


def nerf_matrix_to_ngp(m, scale=NERF_SCALE, offset=(0.5, 0.5, 0.5)):
    """NeRF camera-to-world (3x4 or 4x4) -> ngp mat4x3 as [3 rows, 4 columns] (nerf_loader.h:101-120)."""
    r = np.array(m, np.float32)[:3, :4].copy()
    r[:, 1] *= -1.0
    r[:, 2] *= -1.0
    r[:, 3] = r[:, 3] * scale + np.asarray(offset, np.float32)
    return r[[1, 2, 0], :]   # cycle axes xyz <- yzx


def load_nerf_synthetic(scene_dir, split_json="transforms.json", max_images=None):
    with open(os.path.join(scene_dir, split_json)) as f:
        meta = json.load(f)
    frames = meta["frames"][:max_images] if max_images else meta["frames"]
    images, xforms, focal, pp = [], [], [], []
    for fr in frames:
        path = os.path.join(scene_dir, fr["file_path"])
        if not os.path.splitext(path)[1]:
            path += ".png"
        img = read_png(path)
        h, w = img.shape[:2]
        fx = meta.get("fl_x", 0.5 * w / math.tan(0.5 * meta["camera_angle_x"]))
        fy = meta.get("fl_y", 0.5 * h / math.tan(0.5 * meta["camera_angle_y"])) if ("fl_y" in meta or "camera_angle_y" in meta) else fx
        images.append(img)
        xforms.append(nerf_matrix_to_ngp(fr["transform_matrix"]))
        focal.append((fx, fy))
        pp.append((meta.get("cx", 0.5 * w) / w, meta.get("cy", 0.5 * h) / h))
    return np.stack(images), np.stack(xforms), np.array(focal, np.float32), np.array(pp, np.float32)


def orbit_cameras(n, radius=1.6, center=(0.5, 0.5, 0.5), elevation_deg=(-20.0, 50.0), seed=0):
    """n cameras on a sphere around `center` looking at it (NGP space, [n, 3, 4])."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        az = 2.0 * math.pi * (i + rng.random() * 0.5) / n
        el = math.radians(elevation_deg[0] + (elevation_deg[1] - elevation_deg[0]) * rng.random())
        pos = np.array(center) + radius * np.array([math.cos(el) * math.cos(az), math.sin(el), math.cos(el) * math.sin(az)])
        fwd = np.array(center) - pos
        fwd /= np.linalg.norm(fwd)
        up = np.array([0.0, 1.0, 0.0])
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        out.append(np.stack([right, down, fwd, pos], axis=1).astype(np.float32))   # columns c0 c1 c2 c3
    return np.stack(out)


def render_views(tb, eng, xforms, width, height, fov_deg=40.0):
    """Ground-truth RGBA8 images of the loaded model from the given cameras (instant-NGP Shade render,
    back to 8-bit sRGB with alpha, as a training PNG would hold them)."""
    eng.init(width, height)
    eng.set_param("res_factor", 8)
    tb.set_fov(fov_deg)
    focal = tb.focal_length(0)
    images = []
    for xf in xforms:
        tb.camera_matrix = np.asarray(xf, np.float32).T.reshape(-1)   # column-major 4x3
        r = eng.render_nerf(render_mode=1)
        rgba = r.download("nerf_rgba")
        a = np.clip(rgba[..., 3:4], 0.0, 1.0)
        lin = np.clip(rgba[..., :3], 0.0, None)
        srgb = np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055)
        # shade_kernel_nerf leaves srgb_to_linear(rgb) premultiplied over black: un-premultiply to a PNG-like RGBA
        rgb = np.where(a > 1e-6, srgb / np.maximum(a, 1e-6), 0.0)
        img = np.concatenate([np.clip(rgb, 0, 1), a], axis=-1)
        images.append(np.round(img * 255.0).astype(np.uint8))
    n = len(images)
    return np.stack(images), np.asarray(xforms, np.float32), np.tile(np.asarray(focal, np.float32)[None], (n, 1)), np.full((n, 2), 0.5, np.float32)
