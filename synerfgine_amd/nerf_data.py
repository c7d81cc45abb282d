"""Training data for the online trainer (BASELINE config 5).

* `load_nerf` reads a transforms.json scene with its lens model (read_lens / read_focal_length,
  nerf_loader.cu:175-270), e.g. the reference's real fox capture (OpenCV k1 k2 p1 p2, cx cy).
* `load_nerf_synthetic` reads a NeRF-synthetic scene (transforms.json + 8-bit PNGs, e.g. the lego
  set the reference ships under data/nerf/lego) the way ngp's loader does (nerf_loader.cu:
  focal from fl_x / camera_angle_x, principal point cx/w or 0.5, scale 0.33, offset 0.5, and
  `nerf_matrix_to_ngp`, nerf_loader.h:101-120).
* `render_views` makes a synthetic training set by rendering a model with the instant-NGP
  render path (ground truth for convergence and parity tests without any dataset).
"""
import ctypes
import functools
import json
import math
import os
import re

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


LENS_PERSPECTIVE, LENS_OPENCV, LENS_FTHETA, LENS_LATLONG, LENS_OPENCV_FISHEYE, LENS_EQUIRECTANGULAR = range(6)   # ELensMode (common.h:188-195)


def read_lens(j, lens, principal_point, rolling_shutter):
    """read_lens (nerf_loader.cu:175-239) on one JSON object (the transforms file or a frame): updates
    lens = [mode, params(7)], principal_point = [x, y] (uv) and rolling_shutter = [4] in place."""
    mode = LENS_PERSPECTIVE
    opencv_mode = LENS_OPENCV_FISHEYE if j.get("is_fisheye", False) else LENS_OPENCV
    for name, idx in (("k1", 0), ("k2", 1), ("k3", 2), ("k4", 3), ("p1", 2), ("p2", 3)):
        if name in j:
            lens[1][idx] = float(np.float32(j[name]))
            if lens[1][idx] != 0.0:
                mode = opencv_mode
    if "cx" in j:
        principal_point[0] = float(np.float32(j["cx"]) / np.float32(j["w"]))
    if "cy" in j:
        principal_point[1] = float(np.float32(j["cy"]) / np.float32(j["h"]))
    if "rolling_shutter" in j:
        rs = j["rolling_shutter"]
        rolling_shutter[:] = [float(rs[0]), float(rs[1]), float(rs[2]), float(rs[3]) if len(rs) >= 4 else 0.0]
    if "ftheta_p0" in j:
        for k in range(5):
            lens[1][k] = float(j[f"ftheta_p{k}"])
        lens[1][5], lens[1][6] = float(j["w"]), float(j["h"])
        mode = LENS_FTHETA
    if "latlong" in j:
        mode = LENS_LATLONG
    if "equirectangular" in j:
        mode = LENS_EQUIRECTANGULAR
    if mode != LENS_PERSPECTIVE:   # an outer distortion mode is not overridden by nothing
        lens[0] = mode


_PI_F = np.float32(3.14159265358979323846)   # PI() (random_val.cuh:28), a float


def _tanf(x):
    """glibc's tanf, the function the reference's host-side loader calls (nerf_loader.cu is host code here)."""
    global _libm
    try:
        f = _libm.tanf
    except NameError:
        import ctypes
        import ctypes.util
        _libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _libm.tanf.restype = ctypes.c_float
        _libm.tanf.argtypes = [ctypes.c_float]
        f = _libm.tanf
    return np.float32(f(float(x)))


def _fov_to_focal(res, deg):
    """fov_to_focal_length(int, float) (common_device.cuh:618-620) in float: 0.5f * res / tanf(0.5f * deg * PI() / 180.0f)."""
    f32 = np.float32
    arg = f32(f32(f32(f32(0.5) * f32(deg)) * _PI_F) / f32(180.0))
    return float(f32(f32(0.5) * f32(res)) / _tanf(arg))


def _natural_cmp(a, b):
    """SI::natural::compare (natural_sort.hpp, unvendored; nerf_loader.cu:347-349): runs of digits compare as numbers,
    everything else character by character."""
    ca, cb = [t for t in re.split(r"(\d+)", a) if t], [t for t in re.split(r"(\d+)", b) if t]
    for x, y in zip(ca, cb):
        if x.isdigit() and y.isdigit():
            if int(x) != int(y):
                return -1 if int(x) < int(y) else 1
        elif x != y:
            return -1 if x < y else 1
    return (len(ca) > len(cb)) - (len(ca) < len(cb))


_natural_key = functools.cmp_to_key(_natural_cmp)


def read_focal_length(j, focal, res):
    """read_focal_length (nerf_loader.cu:241-270): per axis x_fov (deg) > fl_x > camera_angle_x (rad); y falls back to x."""
    def axis(r, a):
        if f"{a}_fov" in j:
            return _fov_to_focal(r, float(j[f"{a}_fov"]))
        if f"fl_{a}" in j:
            return float(np.float32(j[f"fl_{a}"]))
        if f"camera_angle_{a}" in j:
            # (float)json["camera_angle_x"] * 180 / PI(): float arithmetic
            return _fov_to_focal(r, np.float32(np.float32(np.float32(j[f"camera_angle_{a}"]) * np.float32(180)) / _PI_F))
        return 0.0
    x, y = axis(res[0], "x"), axis(res[1], "y")
    if x != 0.0:
        focal[0] = focal[1] = x
        if y != 0.0:
            focal[1] = y
    elif y != 0.0:
        focal[0] = focal[1] = y
    else:
        return False
    return True


def load_nerf(scene_dir, split_json="transforms.json", max_images=None):
    """load_nerf (nerf_loader.cu:272-700) for one transforms file of 8-bit PNG images: scale 0.33 / offset 0.5 unless
    the file gives them, aabb_scale, the lens / principal point / rolling shutter of read_lens (the file's, then each
    frame's), the focal length of read_focal_length (the file's, then each frame's), the frames sorted naturally by
    file_path (nerf_loader.cu:347-349), frames kept only when their image
    exists (the sharpness branch, threshold 0 by default, nerf_loader.cu:364-386), nerf_matrix_to_ngp.
    Returns a dict: images [n,h,w,4] u8, xforms [n,3,4], focal [n,2], pp [n,2], lenses [(mode, params)], aabb_scale,
    scale, offset, paths."""
    with open(os.path.join(scene_dir, split_json)) as f:
        meta = json.load(f)
    # the frames in natural order of their file paths, before the n_frames cull and the sharpness filter
    frames = sorted(meta["frames"], key=lambda fr: _natural_key(fr["file_path"].replace("\\", "/")))
    if "n_frames" in meta:
        frames = frames[: min(len(frames), int(meta["n_frames"]))]
    if frames and "sharpness" in frames[0]:
        thr = float(meta.get("sharpness_discard_threshold", 0.0))
        kept = []
        for i, fr in enumerate(frames):
            a, b = max(0, i - 3), min(i + 3, len(frames) - 1)
            mean = sum(float(frames[k].get("sharpness", 1.0)) for k in range(a, b)) / max(1, b - a)
            if os.path.exists(os.path.join(scene_dir, fr["file_path"])) and float(fr.get("sharpness", 1.0)) > thr * mean:
                kept.append(fr)
        frames = kept
    frames = frames[:max_images] if max_images else frames
    scale = float(meta.get("scale", NERF_SCALE))
    off = meta.get("offset", 0.5)
    offset = tuple(float(v) for v in off) if isinstance(off, list) else (float(off),) * 3
    lens0, pp0, rs0 = [LENS_PERSPECTIVE, [0.0] * 7], [0.5, 0.5], [0.0] * 4
    read_lens(meta, lens0, pp0, rs0)
    images, xforms, focal, pp, lenses, paths = [], [], [], [], [], []
    for fr in frames:
        path = os.path.join(scene_dir, fr["file_path"])
        if not os.path.splitext(path)[1]:
            path += ".png"
        img = read_png(path)
        h, w = img.shape[:2]
        fo = [0.0, 0.0]
        got = read_focal_length(meta, fo, (w, h))
        got |= read_focal_length(fr, fo, (w, h))
        if not got:
            raise ValueError(f"{path}: no focal length")
        lens, p, rs = [lens0[0], list(lens0[1])], list(pp0), list(rs0)
        read_lens(fr, lens, p, rs)
        images.append(img)
        xforms.append(nerf_matrix_to_ngp(fr.get("transform_matrix_start", fr["transform_matrix"]), scale, offset))
        focal.append(fo)
        pp.append(p)
        lenses.append((lens[0], lens[1]))
        paths.append(fr["file_path"])
    return {"images": np.stack(images), "xforms": np.stack(xforms), "focal": np.array(focal, np.float32), "pp": np.array(pp, np.float32),
            "lenses": lenses, "aabb_scale": int(meta.get("aabb_scale", 1)), "scale": scale, "offset": offset, "paths": paths}


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
