"""synerfgine_amd -- MI355X-native SyNeRFgine render path.

Host-side mirror of the reference's C++ objects on the hot path, thin over the
C-ABI of libsng_hip.so (include/sng.h):

    Testbed  ~ ngp::Testbed     (load_snapshot, NeRF model, density bitfield, camera,
                                  NerfNetwork::inference_mixed_precision)
    Engine   ~ sng::Engine      (set_virtual_world, init/resize, frame)

All compute runs in the HIP kernels of libsng_hip.so; nothing here falls back
to the CPU.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import SngError, check

__all__ = ["Testbed", "Engine", "FrameResult", "SngError", "device_count"]


def device_count():
    lib = _lib.load()
    n = ctypes.c_int(0)
    check(lib.sng_device_count(ctypes.byref(n)))
    return n.value


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class Testbed:
    """ngp::Testbed subset on the SyNeRFgine path (one context per GPU)."""

    def __init__(self, device_id=0):
        self._lib = _lib.load()
        desc = _lib.sng_ctx_desc(device_id=device_id)
        ctx = ctypes.c_void_p()
        check(self._lib.sng_ctx_create(ctypes.byref(desc), ctypes.byref(ctx)))
        self.ctx = ctx
        self.device_id = device_id

    def close(self):
        if self.ctx:
            check(self._lib.sng_ctx_destroy(self.ctx))
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- model (Testbed::load_snapshot, testbed.cu:4994) -----------------------
    def load_snapshot(self, path):
        check(self._lib.sng_load_snapshot(self.ctx, str(path).encode()))

    def save_snapshot(self, path, include_optimizer_state=False, compress=True):
        """Testbed::save_snapshot (testbed.cu:4812-4876): .ingp = gzip(msgpack), any other suffix = msgpack."""
        check(self._lib.sng_save_snapshot(self.ctx, str(path).encode(), 1 if include_optimizer_state else 0, 1 if compress else 0))

    def set_nerf_model(self, cfg, params):
        params = np.ascontiguousarray(params, dtype=np.float16)
        c = _lib.sng_nerf_config(**cfg)
        check(self._lib.sng_set_nerf_model(self.ctx, ctypes.byref(c), params.view(np.uint16).ctypes.data_as(_lib.U16P), params.size))

    def set_density_grid(self, grid_f16):
        g = np.ascontiguousarray(grid_f16, dtype=np.float16)
        check(self._lib.sng_set_density_grid(self.ctx, g.view(np.uint16).ctypes.data_as(_lib.U16P), g.size))

    def density_grid_bitfield(self):
        out = np.zeros(128 ** 3 // 8 * 8, dtype=np.uint8)
        check(self._lib.sng_get_bitfield(self.ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.size))
        return out

    def density_grid_mean(self):
        v = ctypes.c_float()
        check(self._lib.sng_get_density_mean(self.ctx, ctypes.byref(v)))
        return v.value

    # ---- online training (Testbed::train_nerf, testbed_nerf.cu:3298-3780) ---------
    def set_training_dataset(self, images_rgba8, xforms, focal, principal=None):
        """images [n, h, w, 4] uint8 sRGB; xforms [n, 3, 4] NGP-space camera (columns c0..c3);
        focal [n, 2] in pixels; principal [n, 2] in uv (default 0.5)."""
        im = np.ascontiguousarray(images_rgba8, np.uint8)
        n, h, w, _ = im.shape
        xf = np.ascontiguousarray(np.asarray(xforms, np.float32).reshape(n, 3, 4).transpose(0, 2, 1).reshape(n, 12))   # column-major
        fo = np.ascontiguousarray(np.asarray(focal, np.float32).reshape(n, 2))
        pp = np.ascontiguousarray(np.full((n, 2), 0.5, np.float32) if principal is None else np.asarray(principal, np.float32).reshape(n, 2))
        check(self._lib.sng_train_set_dataset(self.ctx, n, w, h, im.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _fptr(xf), _fptr(fo), _fptr(pp)))

    def set_training_lens(self, lenses):
        """One (mode, params) per training image (read_lens, nerf_loader.cu:175-239; mode 0 Perspective, 1 OpenCV
        {k1 k2 p1 p2}, 2 F-Theta, 3 LatLong, 4 OpenCV fisheye {k1..k4}, 5 Equirectangular); None / [] = all Perspective."""
        if not lenses:
            check(self._lib.sng_train_set_lens(self.ctx, None, 0))
            return
        arr = (_lib.sng_lens * len(lenses))()
        for i, (mode, params) in enumerate(lenses):
            arr[i].mode = int(mode)
            for k, v in enumerate(list(params)[:7]):
                arr[i].params[k] = float(v)
        check(self._lib.sng_train_set_lens(self.ctx, arr, len(lenses)))

    def set_render_lens(self, mode=0, params=()):
        """Testbed::Nerf::render_lens (used while param render_with_lens_distortion is 1); mode 0 = Perspective."""
        l = _lib.sng_lens()
        l.mode = int(mode)
        for k, v in enumerate(list(params)[:7]):
            l.params[k] = float(v)
        check(self._lib.sng_set_render_lens(self.ctx, ctypes.byref(l)))

    def render_lens(self):
        l = _lib.sng_lens()
        check(self._lib.sng_get_render_lens(self.ctx, ctypes.byref(l)))
        return int(l.mode), [float(x) for x in l.params]

    def set_camera_to_training_view(self, view):
        """Testbed::set_camera_to_training_view (testbed.cu:453-469): the training image's camera, focal length,
        principal point and lens (render_with_lens_distortion on)."""
        check(self._lib.sng_set_camera_to_training_view(self.ctx, int(view)))

    def train_reset(self, seed=1337):
        check(self._lib.sng_train_reset(self.ctx, int(seed)))

    def train(self, n_steps):
        st = _lib.sng_train_stats()
        check(self._lib.sng_train(self.ctx, int(n_steps), ctypes.byref(st)))
        out = {k: getattr(st, k) for k in ("step", "loss", "rays_per_batch", "measured_batch", "measured_batch_before_compaction", "ms")}
        if st.timed_steps:   # param train_kernel_times
            out["stage_ms"] = {k: round(getattr(st, "ms_" + k), 5) for k in ("generate", "network", "loss", "grad_clear", "field", "dw", "optimizer")}
        return out

    def training_snapshot(self, n_params, n_cells):
        """(params fp16, density grid fp16) of the trained model -- the .ingp snapshot fields"""
        p = np.zeros(n_params, np.uint16)
        g = np.zeros(n_cells, np.uint16)
        check(self._lib.sng_train_export(self.ctx, p.ctypes.data_as(_lib.U16P), n_params, g.ctypes.data_as(_lib.U16P), n_cells))
        return p.view(np.float16), g.view(np.float16)

    def train_debug(self, stage, name, dtype=np.uint8):
        """parity hook: run the training step up to `stage`, return the named device buffer"""
        n = ctypes.c_uint64()
        check(self._lib.sng_train_debug(self.ctx, int(stage), name.encode(), None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.uint8)
        check(self._lib.sng_train_debug(self.ctx, 0, name.encode(), out.ctypes.data_as(ctypes.c_void_p), out.nbytes, None))
        return out.view(dtype)

    # ---- NerfNetwork::inference_mixed_precision (nerf_network.h:105) -------------
    def inference_mixed_precision(self, d_coords, stride_floats, n, d_out, layout=0, stream=0):
        """Device pointers in, device pointer out (layout 0: tcnn [16][n]; 1: [n][4]; 2: [n][4] density only, NerfNetwork::density)."""
        check(self._lib.sng_nerf_inference(self.ctx, ctypes.c_void_p(d_coords), stride_floats, n, ctypes.c_void_p(d_out), layout,
                                           ctypes.c_void_p(stream)))

    def encode(self, d_coords, stride_floats, n, d_out, stream=0):
        check(self._lib.sng_hashgrid_encode(self.ctx, ctypes.c_void_p(d_coords), stride_floats, n, ctypes.c_void_p(d_out),
                                            ctypes.c_void_p(stream)))

    def sh_encode(self, d_coords, stride_floats, dir_offset, n, d_out, stream=0):
        check(self._lib.sng_sh_encode(self.ctx, ctypes.c_void_p(d_coords), stride_floats, dir_offset, n, ctypes.c_void_p(d_out),
                                      ctypes.c_void_p(stream)))

    # ---- camera (testbed.cu:405-425) ---------------------------------------------
    def set_camera_view(self, view_dir, look_at, scale):
        v = np.asarray(view_dir, np.float32)
        a = np.asarray(look_at, np.float32)
        check(self._lib.sng_set_camera_view(self.ctx, _fptr(v), _fptr(a), float(scale)))

    @property
    def camera_matrix(self):
        m = np.zeros(12, np.float32)
        check(self._lib.sng_get_camera_matrix(self.ctx, _fptr(m)))
        return m

    @camera_matrix.setter
    def camera_matrix(self, m):
        m = np.ascontiguousarray(m, np.float32).ravel()
        check(self._lib.sng_set_camera_matrix(self.ctx, _fptr(m)))

    def set_motion_blur(self, camera1=None, rolling_shutter=None):
        """View::camera1 / rolling_shutter for the NeRF rays (testbed_nerf.cu:1895); None restores the defaults."""
        c1 = None if camera1 is None else np.ascontiguousarray(camera1, np.float32).ravel()
        rs = None if rolling_shutter is None else np.ascontiguousarray(rolling_shutter, np.float32).ravel()
        check(self._lib.sng_set_motion_blur(self.ctx, None if c1 is None else _fptr(c1), None if rs is None else _fptr(rs)))

    def set_fov(self, degrees):
        check(self._lib.sng_set_fov(self.ctx, float(degrees)))

    def focal_length(self, which=0):
        f = np.zeros(2, np.float32)
        check(self._lib.sng_get_focal_length(self.ctx, which, _fptr(f)))
        return f


class FrameResult:
    """sng_frame_result of one frame.  The fields are read from the C struct when first used (a frame loop that does not
    look at them pays no Python time between frames, when the GPU has nothing queued)."""
    _SCALARS = frozenset(("n_iterations", "n_hit", "n_samples", "n_reference_slots", "ms_frame", "ms_raytrace", "ms_nerf", "ms_shadow",
                          "ms_overlay", "ms_network", "network_launches",
                          "fused_from_iter", "n_samples_network", "ms_fused_tail", "n_samples_reused",
                          "onestep_from_iter", "onestep_iterations", "ms_onestep", "onestep_field_evals", "spec_rounds", "spec_evals",
                          "spec_exec", "msr_rounds", "msr_evals", "msr_exec", "sched_reductions"))

    def __init__(self, engine, r):
        self._engine = engine
        self.raw = r

    def __getattr__(self, name):   # only for names not set on the instance
        r = self.__dict__["raw"]
        if name in FrameResult._SCALARS:
            v = getattr(r, name)
        elif name in ("alive_per_iter", "steps_per_iter", "samples_per_iter"):
            v = list(getattr(r, name))[: min(64, r.n_iterations)]
        elif name == "network_launch":
            # per network launch (collect_kernel_times): (samples the launch evaluated, its duration in ms)
            v = [(int(r.samples_network_launch[k]), float(r.ms_network_launch[k])) for k in range(r.n_launch_rec)]
        else:
            raise AttributeError(name)
        self.__dict__[name] = v
        return v

    def download(self, name):
        """Copy a device output buffer to host as float32 [H, W, C]."""
        e = self._engine
        res = e.resolution()
        shapes = {
            "final_rgba": (res["mesh"], 4), "final_depth": (res["mesh"], 1), "syn_rgba": (res["mesh"], 4), "syn_depth": (res["mesh"], 1),
            "nerf_rgba": (res["nerf"], 4), "nerf_depth": (res["nerf"], 1), "nerf_positions": (res["nerf"], 3),
            "nerf_normals": (res["nerf"], 3),
        }
        (w, h), c = shapes[name]
        out = np.empty((h, w, c), np.float32)
        ptr = getattr(self.raw, "d_" + name)
        check(e._lib.sng_copy_to_host(e.ctx, ctypes.c_void_p(ptr), out.ctypes.data_as(ctypes.c_void_p), out.nbytes))
        return out


class Engine:
    """sng::Engine (synerfgine/engine.cu): virtual world, resize and the frame loop."""

    def __init__(self, testbed):
        self.testbed = testbed
        self._lib = testbed._lib
        self.ctx = testbed.ctx

    def set_virtual_world(self, json_path):
        check(self._lib.sng_load_virtual_scene(self.ctx, str(json_path).encode()))

    def init(self, width, height):
        check(self._lib.sng_set_window(self.ctx, int(width), int(height)))
        self._window = (int(width), int(height))

    def set_syn_samples(self, spp):      # --sshadows (engine.cuh:29)
        self.set_param("sshadows", spp)

    def set_nerf_samples(self, k):       # --nshadows (engine.cuh:30-33)
        self.set_param("nshadows", k)

    def set_param(self, key, value):
        check(self._lib.sng_set_param(self.ctx, key.encode(), float(value)))

    def get_param(self, key):
        v = ctypes.c_double()
        check(self._lib.sng_get_param(self.ctx, key.encode(), ctypes.byref(v)))
        return v.value

    def resolution(self):
        r = _lib.sng_resolution_info()
        check(self._lib.sng_get_resolution(self.ctx, ctypes.byref(r)))
        return {"nerf": tuple(r.nerf_res), "mesh": tuple(r.mesh_res), "syn_px_scale": r.syn_px_scale}

    def frame(self, spp=0, reset=True, rows=None, collect_kernel_times=False, target_n_queries=0):
        p = _lib.sng_frame_params(spp=spp, reset_accumulation=1 if reset else 0, collect_kernel_times=1 if collect_kernel_times else 0,
                                  target_n_queries=target_n_queries)
        if rows is not None:
            p.row_begin, p.row_end = rows
        r = _lib.sng_frame_result()
        check(self._lib.sng_render_frame(self.ctx, ctypes.byref(p), ctypes.byref(r)))
        return FrameResult(self, r)

    def frame_buffer(self, name, dtype=np.float32):
        """Debug hook (sng_frame_buffer): a wavefront buffer of the last frame, e.g. "coords"."""
        size = ctypes.c_uint64(0)
        check(self._lib.sng_frame_buffer(self.ctx, name.encode(), None, 0, ctypes.byref(size)))
        out = np.empty(size.value // np.dtype(dtype).itemsize, dtype)
        check(self._lib.sng_frame_buffer(self.ctx, name.encode(), out.ctypes.data_as(ctypes.c_void_p), out.nbytes, None))
        return out

    def rt_counters(self):
        """Traversal counts of the last rt_count = 1 frame: {path, shadow} x {queries, box_tests, tri_tests}."""
        out = (ctypes.c_uint64 * 6)()
        check(self._lib.sng_rt_counters(self.ctx, out))
        keys = ("queries", "box_tests", "tri_tests")
        return {"path": dict(zip(keys, out[0:3])), "shadow": dict(zip(keys, out[3:6]))}

    def render_nerf(self, spp=0, reset=True, rows=None, render_mode=None, collect_kernel_times=False, target_n_queries=0):
        """Testbed::render_nerf: the instant-NGP tracer (composite_kernel_nerf + shade_kernel_nerf), NeRF only."""
        if render_mode is not None:
            self.set_param("render_mode", render_mode)
        p = _lib.sng_frame_params(spp=spp, reset_accumulation=1 if reset else 0, collect_kernel_times=1 if collect_kernel_times else 0,
                                  target_n_queries=target_n_queries)
        if rows is not None:
            p.row_begin, p.row_end = rows
        r = _lib.sng_frame_result()
        check(self._lib.sng_render_nerf_ngp(self.ctx, ctypes.byref(p), ctypes.byref(r)))
        return FrameResult(self, r)

    # ---- multi-GPU step schedule (include/sng.h) ------------------------
    def attach_comm(self, group=None):
        """RCCL communicator over the ranks of `group` (torch.distributed) for the frame-wide step
        schedule: rank 0 makes the ncclUniqueId, the other ranks receive it by broadcast."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = (ctypes.c_uint8 * _lib.SNG_COMM_ID_BYTES)()
        if rank == 0:
            check(self._lib.sng_comm_unique_id(uid))
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=dev)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_uint8 * _lib.SNG_COMM_ID_BYTES)(*t.cpu().tolist())
        check(self._lib.sng_set_comm(self.ctx, uid, rank, world))

    def attach_host_reducer(self, reduce_fn):
        """Host-side schedule exchange: reduce_fn(list_of_ints) -> list of the sums over ranks
        (e.g. a gloo all_reduce); called once per wavefront iteration."""
        def cb(values, n, user):
            try:
                out = reduce_fn([values[i] for i in range(n)])
                for i in range(n):
                    values[i] = int(out[i])
                return 0
            except Exception:   # reported through sng_last_error as "schedule reducer failed"
                return 1
        self._reduce_cb = _lib.SCHED_REDUCE_FN(cb)   # keep alive while attached
        check(self._lib.sng_set_sched_reducer(self.ctx, ctypes.cast(self._reduce_cb, ctypes.c_void_p), None))

    def gather_rgba8(self, bounds, d_frame=0, stream=0):
        """Final composition over the attached RCCL communicator (sng_gather_rgba8): this rank's final rows
        [bounds[rank], bounds[rank+1]) as RGBA8 go to rank 0, straight into d_frame (rank 0: device pointer of
        a height x width uint32 buffer).  Enqueued on `stream` (0: the context's)."""
        b = (ctypes.c_int32 * len(bounds))(*[int(x) for x in bounds])
        check(self._lib.sng_gather_rgba8(self.ctx, b, ctypes.c_void_p(int(d_frame) or None), ctypes.c_void_p(int(stream) or None)))

    def record_schedule(self):
        """A world-size-1 host reducer that records every reduced array of the following frames (sng_set_sched_replay's
        record format); returns the list the records are appended to, as [[n, v0, .., vn-1], ...]."""
        log = []

        def rec(vals):
            log.append([len(vals)] + [int(v) for v in vals])
            return vals
        self.attach_host_reducer(rec)
        return log

    def set_sched_replay(self, records):
        """Replay the reduced arrays `records` ([[n, v...], ...], one frame's reductions in call order) at every
        reduction point of the following frames (sng_set_sched_replay); None detaches."""
        if records is None:
            check(self._lib.sng_set_sched_replay(self.ctx, None, 0))
            return
        flat = np.ascontiguousarray([w for r in records for w in r], np.uint32)
        check(self._lib.sng_set_sched_replay(self.ctx, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), flat.size))

    def detach_comm(self):
        check(self._lib.sng_set_comm(self.ctx, None, 0, 0))
        check(self._lib.sng_set_sched_reducer(self.ctx, None, None))
        check(self._lib.sng_set_sched_replay(self.ctx, None, 0))
        self._reduce_cb = None

    # ---- headless display stage (Display::present / save_image, display.cu:265-322) ----------
    def display(self):
        """The window image of the last frame: main.frag FXAA + clear-colour blend, RGB8 [h][w][3], top-down."""
        w, h = self._window
        out = np.zeros((h, w, 3), np.uint8)
        check(self._lib.sng_display_frame(self.ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.nbytes))
        return out

    def save_image(self, folder=None):
        """Display::save_image: <folder>/output-NNN.png; False once output.img_count is exceeded."""
        w = ctypes.c_int32()
        check(self._lib.sng_save_image(self.ctx, None if folder is None else str(folder).encode(), ctypes.byref(w)))
        return bool(w.value)

    # ---- scene inspection (tests) --------------------------------------------------
    def scene(self):
        no, nl, nm = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self._lib.sng_get_scene_counts(self.ctx, ctypes.byref(no), ctypes.byref(nl), ctypes.byref(nm)))
        objs = []
        for i in range(no.value):
            info = _lib.sng_object_info()
            check(self._lib.sng_get_object(self.ctx, i, ctypes.byref(info)))
            nodes = np.zeros((info.n_nodes, 8), np.float32)
            tris = np.zeros((info.n_tris, 9), np.float32)
            check(self._lib.sng_get_object_bvh(self.ctx, i, _fptr(nodes), _fptr(tris)))
            objs.append(dict(nodes=nodes, tris=tris, rot=np.array(info.rot, np.float32), pos=np.array(info.pos, np.float32),
                             scale=info.scale, mat_id=info.mat_id))
        lights = []
        for i in range(nl.value):
            l = _lib.sng_light()
            check(self._lib.sng_get_light(self.ctx, i, ctypes.byref(l)))
            lights.append(dict(pos=list(l.pos), intensity=l.intensity, size=l.size, type=l.type))
        mats = []
        for i in range(nm.value):
            m = _lib.sng_material()
            check(self._lib.sng_get_material(self.ctx, i, ctypes.byref(m)))
            mats.append(dict(ka=list(m.ka), kd=list(m.kd), ks=list(m.ks), n=m.n, rg=m.rg, spec_angle=m.spec_angle, type=m.type))
        return objs, lights, mats

    def rng_states(self, which):
        res = self.resolution()
        w, h = res["nerf"] if which == 0 else res["mesh"]
        out = np.zeros((w * h, 6), np.uint32)
        check(self._lib.sng_get_rng_states(self.ctx, which, out.ctypes.data_as(_lib.U32P), w * h))
        return out

    def set_rng_states(self, which, states):
        states = np.ascontiguousarray(states, np.uint32)
        check(self._lib.sng_set_rng_states(self.ctx, which, states.ctypes.data_as(_lib.U32P), states.shape[0]))


def write_png(path, image):
    """uint8 [h][w][3|4] -> PNG (host; the recording's stbi_write_png)."""
    im = np.ascontiguousarray(image, np.uint8)
    check(_lib.load().sng_image_write_png(str(path).encode(), im.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), im.shape[1], im.shape[0],
                                          im.shape[2]))


def animation_probe(scene_json, n_frames, playing=None, animation_speed=None, max_lights=64, max_objects=64):
    """Host-only (no device): play a scene JSON's animation for n_frames in Engine::frame's order --
    (cameras [n][3][4], light positions [n][L][3], object positions [n][O][3])."""
    lib = _lib.load()
    cams = np.zeros((n_frames, 12), np.float32)
    lp = np.zeros((n_frames, max_lights, 3), np.float32)
    op = np.zeros((n_frames, max_objects, 3), np.float32)
    nl, no = ctypes.c_uint32(), ctypes.c_uint32()
    check(lib.sng_animation_probe(str(scene_json).encode(), n_frames, -1 if playing is None else int(bool(playing)),
                                  -1.0 if animation_speed is None else float(animation_speed), _fptr(cams), _fptr(lp), max_lights, _fptr(op),
                                  max_objects, ctypes.byref(nl), ctypes.byref(no)))
    L, O = nl.value, no.value
    lp = lp.reshape(-1)[: n_frames * L * 3].reshape(n_frames, L, 3)
    op = op.reshape(-1)[: n_frames * O * 3].reshape(n_frames, O, 3)
    return cams.reshape(n_frames, 4, 3).transpose(0, 2, 1), lp, op


def bvh_build(tris, prims_per_leaf=4):
    """TriangleBvhWithBranchingFactor<2>::build on the host (A13). Returns (nodes [n,8], reordered tris)."""
    lib = _lib.load()
    t = np.ascontiguousarray(tris, np.float32).reshape(-1, 9).copy()
    cap = 4 * t.shape[0] + 8
    nodes = np.zeros((cap, 8), np.float32)
    n = ctypes.c_uint32()
    check(lib.sng_bvh_build(_fptr(t), t.shape[0], prims_per_leaf, _fptr(nodes), cap, ctypes.byref(n)))
    return nodes[: n.value], t
