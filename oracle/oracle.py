"""ctypes binding of the CPU ORACLE (oracle/_build/libsng_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.  See
oracle/sng_oracle.h for the parity status (partially pinned).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libsng_oracle.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class orc_model(ctypes.Structure):
    _fields_ = [("n_levels", ctypes.c_uint32), ("n_features", ctypes.c_uint32), ("log2_hashmap_size", ctypes.c_uint32),
                ("base_resolution", ctypes.c_uint32), ("per_level_scale", ctypes.c_float), ("params", ctypes.c_void_p)]


class orc_volume(ctypes.Structure):
    _fields_ = [("render_aabb_min", ctypes.c_float * 3), ("render_aabb_max", ctypes.c_float * 3),
                ("train_aabb_min", ctypes.c_float * 3), ("train_aabb_max", ctypes.c_float * 3),
                ("render_aabb_to_local", ctypes.c_float * 9), ("cone_angle_constant", ctypes.c_float),
                ("max_mip", ctypes.c_uint32), ("min_transmittance", ctypes.c_float), ("bitfield", ctypes.c_void_p)]


class orc_camera(ctypes.Structure):
    _fields_ = [("camera", ctypes.c_float * 12), ("focal", ctypes.c_float * 2), ("screen_center", ctypes.c_float * 2),
                ("res", ctypes.c_int32 * 2), ("spp", ctypes.c_uint32), ("snap_to_pixel_centers", ctypes.c_int32),
                ("target_n_queries", ctypes.c_uint32)]


class orc_object(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_void_p), ("tris", ctypes.c_void_p), ("rot", ctypes.c_float * 9), ("pos", ctypes.c_float * 3),
                ("scale", ctypes.c_float), ("mat_id", ctypes.c_int32)]


class orc_light(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 3), ("intensity", ctypes.c_float), ("size", ctypes.c_float), ("type", ctypes.c_int32)]


class orc_material(ctypes.Structure):
    _fields_ = [("ka", ctypes.c_float * 3), ("kd", ctypes.c_float * 3), ("ks", ctypes.c_float * 3), ("n", ctypes.c_float),
                ("rg", ctypes.c_float), ("spec_angle", ctypes.c_float), ("type", ctypes.c_int32)]


class orc_train_images(ctypes.Structure):
    _fields_ = [("rgba", ctypes.c_void_p), ("xforms", ctypes.c_void_p), ("focal", ctypes.c_void_p), ("pp", ctypes.c_void_p),
                ("w", ctypes.c_int32), ("h", ctypes.c_int32), ("n", ctypes.c_int32)]


class orc_keyframe(ctypes.Structure):
    _fields_ = [("view", ctypes.c_float * 3), ("at", ctypes.c_float * 3), ("zoom", ctypes.c_float)]


class orc_light_anim(ctypes.Structure):
    _fields_ = [("on", ctypes.c_int32), ("start", ctypes.c_float * 3), ("end", ctypes.c_float * 3), ("ratio", ctypes.c_float),
                ("step", ctypes.c_float)]


class orc_object_anim(ctypes.Structure):
    _fields_ = [("angle", ctypes.c_float), ("axis", ctypes.c_float * 3), ("centre", ctypes.c_float * 3), ("rot", ctypes.c_float * 9),
                ("pos", ctypes.c_float * 3)]


class orc_nerf_stats(ctypes.Structure):
    _fields_ = [("n_iterations", ctypes.c_uint32), ("n_samples", ctypes.c_uint64), ("n_slots", ctypes.c_uint64),
                ("n_hit", ctypes.c_uint32), ("alive_per_iter", ctypes.c_uint32 * 64), ("steps_per_iter", ctypes.c_uint32 * 64)]


class orc_frame_params(ctypes.Structure):
    _fields_ = [("nerf_res", ctypes.c_int32 * 2), ("mesh_res", ctypes.c_int32 * 2), ("syn_px_scale", ctypes.c_int32),
                ("show_nerf", ctypes.c_int32), ("show_virtual_obj", ctypes.c_int32), ("shadow_on_nerf", ctypes.c_int32),
                ("shadow_on_virtual_obj", ctypes.c_int32), ("nerf_shadow_intensity", ctypes.c_float),
                ("nerf_on_nerf_shadow_threshold", ctypes.c_float), ("nerf_kernel_size", ctypes.c_int32),
                ("light_samples", ctypes.c_uint32), ("path_trace_depth", ctypes.c_uint32), ("shadow_iters", ctypes.c_uint32),
                ("shadow_steps", ctypes.c_uint32), ("lens_angle_constant", ctypes.c_float), ("syn_shadow_factor", ctypes.c_float),
                ("rt_depth_offset", ctypes.c_float), ("exposure", ctypes.c_float), ("srgb_output", ctypes.c_int32),
                ("tonemap_curve", ctypes.c_int32), ("rt_buffer_type", ctypes.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        u32, u64, f32, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float, ctypes.c_int32
        sig = {
            "orc_morton3D": (u32, [u32, u32, u32]), "orc_morton3D_invert": (u32, [u32]), "orc_sobol": (u32, [u32, u32]),
            "orc_ld_random_val": (f32, [u32, u32, u32]), "orc_ld_random_pixel_offset": (None, [u32, vp]),
            "orc_float_to_half": (ctypes.c_uint16, [f32]), "orc_half_to_float": (f32, [ctypes.c_uint16]),
            "orc_xorwow_init": (None, [u64, u64, u64, vp]), "orc_xorwow_init_many": (None, [u64, u32, vp]),
            "orc_xorwow_next": (u32, [vp]), "orc_curand_uniform": (f32, [vp]),
            "orc_xorwow_jump_steps_naive": (None, [vp, u64]), "orc_xorwow_jump_matrix": (None, [vp, u32]),
            "orc_grid_level_table": (u32, [vp, vp, vp]), "orc_n_params": (u32, [vp]),
            "orc_hashgrid_encode": (None, [vp, vp, u32, u32, vp]), "orc_sh_encode": (None, [vp, u32, u32, u32, vp]),
            "orc_nerf_inference": (None, [vp, vp, u32, u32, vp]),
            "orc_wavefront_schedule": (None, [vp, u32, u32, vp, vp]),
            "orc_density_grid_to_bitfield": (None, [vp, u32, vp, vp]),
            "orc_render_nerf": (None, [vp, vp, vp, vp, vp, vp, vp, vp]),
            "orc_render_nerf_ngp": (None, [vp, vp, vp, i32, f32, vp, vp, vp]),
            "orc_shade_nerf_shadows": (None, [vp, vp, vp, vp, vp, vp, u32, vp, u32, vp, f32, f32, i32]),
            "orc_bvh_build": (i32, [vp, u32, u32, vp, u32]),
            "orc_depth_test_world": (None, [vp, u32, vp, vp, u32, vp, vp]),
            "orc_mesh_init_rays": (None, [vp, vp, vp, vp, vp]),
            "orc_raytrace": (None, [vp, vp, vp, vp, u32, vp, u32, vp, u32, vp, vp, u32, vp, vp, vp]),
            "orc_overlay": (None, [vp, vp, vp, vp, vp, vp, vp]),
            "orc_render_frame": (None, [vp, vp, vp, vp, vp, vp, u32, vp, u32, vp, u32, vp, vp, vp, vp, vp, vp, vp]),
            "orc_num_threads": (i32, []), "orc_set_num_threads": (None, [i32]), "orc_set_mlp_accum": (None, [i32, i32]),
            "orc_set_visualization": (None, [i32, i32]),
            "orc_set_motion_blur": (None, [vp, vp]), "orc_set_glow": (None, [i32, f32]), "orc_set_shadow_rng_mode": (None, [i32]), "orc_set_literal": (None, [i32]),
            "orc_set_gbuffer_out": (None, [vp, vp]),
            "orc_set_render_lens": (None, [vp]), "orc_set_train_lens": (None, [vp, u32]),
            "orc_uv_to_ray_dir": (i32, [vp, vp, i32, i32, vp, vp, vp]), "orc_lens_distortion_delta": (None, [vp, f32, f32, vp, vp]),
            "orc_train_generate": (None, [vp, vp, u64, u64, u32, u32, vp, vp, vp]),
            "orc_display": (None, [vp, i32, i32, i32, i32, vp, vp]),
            "orc_camera_set_view": (None, [vp, vp, vp, vp, vp, f32]),
            "orc_animation_play": (None, [vp, vp, vp, vp, u32, i32, i32, f32, vp, u32, vp, u32, u32, vp, vp, vp]),
            "orc_train_adam_ema": (None, [u64, u32, f32, f32, f32, f32, f32, f32, f32, u32, vp, vp, vp, vp, vp, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


class literal:
    """Context manager: the oracle evaluates the reference's text as written (on = 1, the default) or the product's
    restatements of its --use_fast_math build (on = 0: reciprocal-multiply box tests, integer powers by binary
    exponentiation, the clamped overlay index; orc_set_literal, sng_oracle.h)."""
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        lib().orc_set_literal(1 if self.on else 0)
        return self

    def __exit__(self, *exc):
        lib().orc_set_literal(1)
        return False


class mlp_accum:
    """Context manager: run the oracle MLP with tcnn's fp16 WMMA accumulators (mode 1) or fp32 (mode 0)."""
    def __init__(self, mode, chunk=16):
        self.mode, self.chunk = mode, chunk

    def __enter__(self):
        lib().orc_set_mlp_accum(self.mode, self.chunk)
        return self

    def __exit__(self, *exc):
        lib().orc_set_mlp_accum(0, 16)
        return False


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class motion_blur:
    """Context manager: NeRF camera rays with View::camera1 / rolling_shutter (testbed_nerf.cu:1895)."""
    def __init__(self, camera1=None, rolling_shutter=None):
        self.c1 = None if camera1 is None else np.ascontiguousarray(np.asarray(camera1, np.float32).ravel())
        self.rs = None if rolling_shutter is None else np.ascontiguousarray(rolling_shutter, np.float32)

    def __enter__(self):
        lib().orc_set_motion_blur(None if self.c1 is None else ptr(self.c1), None if self.rs is None else ptr(self.rs))
        return self

    def __exit__(self, *exc):
        lib().orc_set_motion_blur(None, None)
        return False


# ---- convenience wrappers -----------------------------------------------------------
class Model:
    def __init__(self, cfg, params):
        self.params = np.ascontiguousarray(params, np.float16)
        self.s = orc_model(cfg["n_levels"], cfg["n_features_per_level"], cfg["log2_hashmap_size"], cfg["base_resolution"],
                           cfg["per_level_scale"], self.params.ctypes.data)

    def ref(self):
        return ctypes.byref(self.s)


def level_table(cfg):
    m = Model(cfg, np.zeros(1, np.float16))
    offs = np.zeros(cfg["n_levels"] + 1, np.uint32)
    res = np.zeros(cfg["n_levels"], np.uint32)
    lib().orc_grid_level_table(m.ref(), ptr(offs), ptr(res))
    return offs, res


def encode(model, coords, stride):
    n = coords.size // stride
    out = np.zeros((n, 32), np.uint16)
    lib().orc_hashgrid_encode(model.ref(), ptr(np.ascontiguousarray(coords, np.float32)), stride, n, ptr(out))
    return out.view(np.float16)


def inference(model, coords, stride=7):
    c = np.ascontiguousarray(coords, np.float32)
    n = c.size // stride
    out = np.zeros((n, 16), np.uint16)
    lib().orc_nerf_inference(model.ref(), ptr(c), stride, n, ptr(out))
    return out.view(np.float16)


def bitfield(grid_f16, max_cascade=0):
    g = np.ascontiguousarray(grid_f16, np.float16)
    bf = np.zeros(128 ** 3 // 8 * 8, np.uint8)
    mean = ctypes.c_float()
    lib().orc_density_grid_to_bitfield(ptr(g.view(np.uint16)), max_cascade, ptr(bf), ctypes.byref(mean))
    return bf, mean.value


def xorwow_states(n, seed=1999):
    st = np.zeros((n, 6), np.uint32)
    lib().orc_xorwow_init_many(seed, n, ptr(st))
    return st


def volume_for(cfg, grid_f16, min_transmittance=0.01):
    """Bitfield + volume of a model config (aabb_scale -> max_cascade, cone) from its density grid."""
    a = int(cfg.get("aabb_scale", 1))
    mc = 0
    while (1 << mc) < a:
        mc += 1
    bf, _ = bitfield(grid_f16, max_cascade=mc)
    return make_volume(bf, aabb_scale=a, min_transmittance=min_transmittance)


def make_volume(bf, aabb_scale=1, min_transmittance=0.01):
    h = 0.5 * min(128, aabb_scale)
    lo, hi = [0.5 - h] * 3, [0.5 + h] * 3
    mc = 0
    while (1 << mc) < aabb_scale:
        mc += 1
    v = orc_volume()
    v.render_aabb_min[:] = lo; v.render_aabb_max[:] = hi
    v.train_aabb_min[:] = lo; v.train_aabb_max[:] = hi
    v.render_aabb_to_local[:] = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    v.cone_angle_constant = 0.0 if aabb_scale <= 1 else 1.0 / 256.0
    v.max_mip = mc
    v.min_transmittance = min_transmittance
    v._bf = bf
    v.bitfield = bf.ctypes.data
    return v


def make_camera(matrix, focal, res, spp=0, screen_center=(0.5, 0.5), target=0):
    c = orc_camera()
    c.camera[:] = list(np.asarray(matrix, np.float32).ravel())
    c.focal[:] = list(focal)
    c.screen_center[:] = list(screen_center)
    c.res[:] = list(res)
    c.spp = spp
    c.snap_to_pixel_centers = 0
    c.target_n_queries = target
    return c


def make_objects(objs):
    arr = (orc_object * max(1, len(objs)))()
    keep = []
    for i, o in enumerate(objs):
        nodes = np.ascontiguousarray(o["nodes"], np.float32)
        tris = np.ascontiguousarray(o["tris"], np.float32)
        keep += [nodes, tris]
        arr[i].nodes = nodes.ctypes.data
        arr[i].tris = tris.ctypes.data
        arr[i].rot[:] = list(np.asarray(o["rot"], np.float32))
        arr[i].pos[:] = list(np.asarray(o["pos"], np.float32))
        arr[i].scale = o["scale"]
        arr[i].mat_id = o["mat_id"]
    arr._keep = keep
    return arr


def make_lights(lights):
    arr = (orc_light * max(1, len(lights)))()
    for i, l in enumerate(lights):
        arr[i].pos[:] = l["pos"]; arr[i].intensity = l["intensity"]; arr[i].size = l["size"]; arr[i].type = l["type"]
    return arr


def make_materials(mats):
    arr = (orc_material * max(1, len(mats)))()
    for i, m in enumerate(mats):
        arr[i].ka[:] = m["ka"]; arr[i].kd[:] = m["kd"]; arr[i].ks[:] = m["ks"]
        arr[i].n = m["n"]; arr[i].rg = m["rg"]; arr[i].spec_angle = m["spec_angle"]; arr[i].type = m["type"]
    return arr


def render_nerf(model, vol, cam):
    W, H = cam.res[0], cam.res[1]
    rgba = np.zeros((H, W, 4), np.float32)
    depth = np.zeros((H, W), np.float32)
    pos = np.zeros((H, W, 3), np.float32)
    nrm = np.zeros((H, W, 3), np.float32)
    st = orc_nerf_stats()
    lib().orc_render_nerf(model.ref(), ctypes.byref(vol), ctypes.byref(cam), ptr(rgba), ptr(depth), ptr(pos), ptr(nrm), ctypes.byref(st))
    return rgba, depth, pos, nrm, st


def render_nerf_ngp(model, vol, cam, render_mode=1, depth_scale=1.0, vis_layer=0, vis_dim=0, glow_mode=0, glow_y_cutoff=0.0):
    """instant-NGP render path (A22): returns rgba [H,W,4], depth [H,W], stats."""
    W, H = cam.res[0], cam.res[1]
    rgba = np.zeros((H, W, 4), np.float32)
    depth = np.zeros((H, W), np.float32)
    st = orc_nerf_stats()
    lib().orc_set_visualization(vis_layer, vis_dim)
    lib().orc_set_glow(glow_mode, glow_y_cutoff)
    try:
        lib().orc_render_nerf_ngp(model.ref(), ctypes.byref(vol), ctypes.byref(cam), render_mode, depth_scale, ptr(rgba), ptr(depth), ctypes.byref(st))
    finally:
        lib().orc_set_glow(0, 0.0)
    return rgba, depth, st


def frame_params_from_engine(eng):
    """orc_frame_params mirroring the Engine/RayTracer parameters of a product engine."""
    r = eng.resolution()
    p = orc_frame_params()
    p.nerf_res[:] = list(r["nerf"]); p.mesh_res[:] = list(r["mesh"]); p.syn_px_scale = r["syn_px_scale"]
    g = eng.get_param
    p.show_nerf = int(g("show_nerf")); p.show_virtual_obj = int(g("show_virtual_obj"))
    p.shadow_on_nerf = int(g("shadow_on_nerf")); p.shadow_on_virtual_obj = int(g("shadow_on_virtual_obj"))
    p.nerf_shadow_intensity = g("nerf_shadow_intensity"); p.nerf_on_nerf_shadow_threshold = g("nerf_on_nerf_shadow_threshold")
    p.nerf_kernel_size = int(g("nerf_shadow_samples")); p.light_samples = int(g("light_samples"))
    p.path_trace_depth = int(g("path_trace_depth")); p.shadow_iters = int(g("syn_shadow_samples")); p.shadow_steps = int(g("n_steps"))
    p.lens_angle_constant = g("lens_size"); p.syn_shadow_factor = g("syn_shadow_intensity"); p.rt_depth_offset = g("depth_offset")
    p.exposure = g("exposure"); p.srgb_output = int(g("srgb")); p.tonemap_curve = int(g("tonemap_curve"))
    p.rt_buffer_type = int(g("rt_buffer_type"))
    return p


def render_frame(model, vol, tb, eng, nerf_rng, mesh_rng, spp=0, target=0, gbuffer=False):
    """Whole Engine::frame on the CPU with the product's camera/scene/RNG inputs (rng arrays are advanced in place)."""
    r = eng.resolution()
    cam = tb.camera_matrix
    ncam = make_camera(cam, tb.focal_length(0), r["nerf"], spp=spp, target=target)
    mcam = make_camera(cam, tb.focal_length(1), r["mesh"], spp=spp, target=target)
    p = frame_params_from_engine(eng)
    objs, lights, mats = eng.scene()
    oo, ll, mm = make_objects(objs), make_lights(lights), make_materials(mats)
    (mw, mh), (nw, nh) = r["mesh"], r["nerf"]
    final = np.zeros((mh, mw, 4), np.float32); final_d = np.zeros((mh, mw), np.float32)
    nrgba = np.zeros((nh, nw, 4), np.float32); ndepth = np.zeros((nh, nw), np.float32)
    st = orc_nerf_stats()
    gpos = gnrm = None
    if gbuffer:
        gpos, gnrm = np.zeros((nh, nw, 3), np.float32), np.zeros((nh, nw, 3), np.float32)
        lib().orc_set_gbuffer_out(ptr(gpos), ptr(gnrm))
    lib().orc_render_frame(model.ref(), ctypes.byref(vol), ctypes.byref(ncam), ctypes.byref(mcam), ctypes.byref(p), ctypes.addressof(oo),
                           len(objs), ctypes.addressof(ll), len(lights), ctypes.addressof(mm), len(mats), ptr(nerf_rng), ptr(mesh_rng), ptr(final), ptr(final_d), ptr(nrgba), ptr(ndepth),
                           ctypes.byref(st))
    if gbuffer:
        lib().orc_set_gbuffer_out(None, None)
    return dict(final=final, final_depth=final_d, nerf_rgba=nrgba, nerf_depth=ndepth, stats=st, positions=gpos, normals=gnrm)


# ---- online training (config 5) ----------------------------------------------------
class orc_lens(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("params", ctypes.c_float * 7)]


def _lens_array(lenses):
    """[(mode, params...), ...] -> ctypes array of orc_lens (params padded to 7)"""
    arr = (orc_lens * max(1, len(lenses)))()
    for i, (mode, params) in enumerate(lenses):
        arr[i].mode = int(mode)
        for k, v in enumerate(list(params)[:7]):
            arr[i].params[k] = float(v)
    return arr


def set_render_lens(mode=0, params=()):
    """the NeRF camera rays' lens (Testbed::Nerf::render_lens with render_with_lens_distortion); mode 0 = Perspective"""
    lib().orc_set_render_lens(ctypes.byref(_lens_array([(mode, params)])[0]) if mode else None)


def uv_to_ray_dir(lens, uv, res, focal, screen_center):
    """uv_to_ray's camera-space direction (valid, dir[3]) for lens = (mode, params)"""
    arr = _lens_array([lens])
    u = np.asarray(uv, np.float32)
    f = np.asarray(focal, np.float32)
    sc = np.asarray(screen_center, np.float32)
    d = np.zeros(3, np.float32)
    ok = lib().orc_uv_to_ray_dir(ctypes.byref(arr[0]), u.ctypes.data, int(res[0]), int(res[1]), f.ctypes.data, sc.ctypes.data, d.ctypes.data)
    return bool(ok), d


def lens_distortion_delta(lens, u, v):
    arr = _lens_array([lens])
    du, dv = ctypes.c_float(), ctypes.c_float()
    lib().orc_lens_distortion_delta(ctypes.byref(arr[0]), float(u), float(v), ctypes.byref(du), ctypes.byref(dv))
    return du.value, dv.value


def set_train_lens(lenses):
    """one (mode, params) per training image for train_generate; [] = all Perspective"""
    arr = _lens_array(lenses)
    lib().orc_set_train_lens(arr, len(lenses))


def train_generate(vol, images, xforms, focal, pp, rng_state, rng_inc, n_rays, max_per_ray=1024):
    """generate_training_samples_nerf for rays [0, n_rays): (numsteps [n], rays [n][6], coords [n][max_per_ray][7]).
    images [n, h, w, 4] uint8; xforms [n, 3, 4] NGP camera (columns c0..c3); the lenses of set_train_lens."""
    im = np.ascontiguousarray(images, np.uint8)
    xf = np.ascontiguousarray(np.asarray(xforms, np.float32).reshape(-1, 3, 4).transpose(0, 2, 1).reshape(-1, 12))
    fo = np.ascontiguousarray(focal, np.float32)
    p = np.ascontiguousarray(pp, np.float32)
    desc = orc_train_images(im.ctypes.data, xf.ctypes.data, fo.ctypes.data, p.ctypes.data, im.shape[2], im.shape[1], im.shape[0])
    ns = np.zeros(n_rays, np.uint32)
    rays = np.zeros((n_rays, 6), np.float32)
    co = np.zeros((n_rays, max_per_ray, 7), np.float32)
    lib().orc_train_generate(ctypes.byref(vol), ctypes.byref(desc), rng_state, rng_inc, n_rays, max_per_ray, ptr(ns), ptr(rays), ptr(co))
    return ns, rays, co


def train_adam_ema(master, grads, m1, m2, steps, ema, n_matrix, lr=1e-2, beta1=0.9, beta2=0.99, eps=1e-15, l2_reg=1e-6, loss_scale=128.0,
                   ema_decay=0.95, ema_step=0):
    """One Ema(Adam) step in place on float32 / uint32 arrays."""
    for a, dt in ((master, np.float32), (grads, np.float32), (m1, np.float32), (m2, np.float32), (steps, np.uint32), (ema, np.float32)):
        assert a.dtype == dt and a.flags.c_contiguous
    lib().orc_train_adam_ema(len(master), n_matrix, lr, beta1, beta2, eps, l2_reg, loss_scale, ema_decay, ema_step, ptr(master), ptr(grads),
                             ptr(m1), ptr(m2), ptr(steps), ptr(ema))


# ---- scene animation (camera path, lights, objects) ---------------------------------
TESTBED_DEFAULT_CAMERA = [1, 0, 0, 0, -1, 0, 0, 0, -1, 0.5, 0.5, 2.0]   # Testbed::reset_camera (testbed.cu:470-490)
TESTBED_DEFAULT_SCALE = 1.5


def animation_play(scene, n_frames, playing=None, anim_speed=None):
    """Play a parsed scene JSON's animation: (cameras [n][12], light positions [n][L][3], object positions [n][O][3])."""
    cam = np.array(TESTBED_DEFAULT_CAMERA, np.float32)
    scale = ctypes.c_float(TESTBED_DEFAULT_SCALE)
    up = np.array([0, 1, 0], np.float32)
    cc = scene.get("camera", {})
    view = np.array(cc.get("view", [0, 0, 0]), np.float32)
    if np.dot(view, view) != 0:
        lib().orc_camera_set_view(ptr(cam), ctypes.byref(scale), ptr(up), ptr(view), ptr(np.array(cc.get("at", [0, 0, 0]), np.float32)),
                                  float(cc.get("zoom", 1.0)))
    keys = []
    if "path" in cc:
        keys = list(cc.get("frames", [])) + list(cc["path"])
    kk = (orc_keyframe * max(1, len(keys)))()
    for i, k in enumerate(keys):
        kk[i].view[:] = k["view"]; kk[i].at[:] = k["at"]; kk[i].zoom = k["zoom"]
    total = int(cc.get("total_time_ms", 10000)) * int(cc.get("fps", 24)) // 1000
    play = bool(cc.get("move_on_start", False)) if playing is None else bool(playing)
    speed = float(cc.get("animation_speed", 0.0)) if anim_speed is None else float(anim_speed)
    ls = scene.get("lights", [])
    la = (orc_light_anim * max(1, len(ls)))()
    for i, l in enumerate(ls):
        la[i].start[:] = l["pos"]
        if "anim" in l:
            la[i].on = 1; la[i].end[:] = l["anim"]["end"]; la[i].step = l["anim"]["step"]
    os_ = scene.get("objfile", [])
    oa = (orc_object_anim * max(1, len(os_)))()
    for i, o in enumerate(os_):
        oa[i].rot[:] = o.get("rot", [1, 0, 0, 0, 1, 0, 0, 0, 1]); oa[i].pos[:] = o.get("pos", [0, 0, 0])
        oa[i].axis[:] = [0, 1, 0]
        if "anim" in o:
            oa[i].angle = o["anim"]["rot_angle"]; oa[i].axis[:] = o["anim"]["rot_axis"]; oa[i].centre[:] = o["anim"]["rot_center"]
    cams = np.zeros((n_frames, 12), np.float32)
    lp = np.zeros((n_frames, len(ls), 3), np.float32)
    op = np.zeros((n_frames, len(os_), 3), np.float32)
    vp = ctypes.c_void_p
    lib().orc_animation_play(ptr(cam), ctypes.byref(scale), ptr(up), ctypes.cast(kk, vp), len(keys), total, int(play), speed, ctypes.cast(la, vp),
                             len(ls), ctypes.cast(oa, vp), len(os_), n_frames, ptr(cams), ptr(lp), ptr(op))
    return cams, lp, op


def display(rgba, out_w=None, out_h=None, clear=(0.0, 0.0, 0.0)):
    """main.frag FXAA + blend + unorm8 of a final RGBA32F frame [h][w][4] -> RGB8 [oh][ow][3]."""
    im = np.ascontiguousarray(rgba, np.float32)
    h, w = im.shape[:2]
    ow, oh = out_w or w, out_h or h
    out = np.zeros((oh, ow, 3), np.uint8)
    cl = np.asarray(clear, np.float32)
    lib().orc_display(ptr(im), w, h, ow, oh, ptr(cl), ptr(out))
    return out
