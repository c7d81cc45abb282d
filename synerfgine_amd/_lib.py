"""ctypes binding of libsng_hip.so (include/sng.h).

The library is the product: hand-written HIP kernels for gfx950 plus the C++
host runtime.  There is no CPU fallback -- if the library is missing the
import fails loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SNG_LIB_PATH") or os.path.join(_HERE, "_build", "libsng_hip.so")   # override: A/B builds (tools/)

SNG_OK = 0


class SngError(RuntimeError):
    pass


class sng_ctx_desc(ctypes.Structure):
    _fields_ = [("device_id", ctypes.c_int32), ("reserved", ctypes.c_int32 * 7)]


class sng_nerf_config(ctypes.Structure):
    _fields_ = [
        ("n_levels", ctypes.c_uint32),
        ("n_features_per_level", ctypes.c_uint32),
        ("log2_hashmap_size", ctypes.c_uint32),
        ("base_resolution", ctypes.c_uint32),
        ("per_level_scale", ctypes.c_float),
        ("aabb_scale", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 6),
    ]


class sng_resolution_info(ctypes.Structure):
    _fields_ = [
        ("nerf_res", ctypes.c_int32 * 2),
        ("mesh_res", ctypes.c_int32 * 2),
        ("syn_px_scale", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 3),
    ]


class sng_frame_params(ctypes.Structure):
    _fields_ = [
        ("spp", ctypes.c_uint32),
        ("reset_accumulation", ctypes.c_int32),
        ("row_begin", ctypes.c_int32),
        ("row_end", ctypes.c_int32),
        ("collect_kernel_times", ctypes.c_int32),
        ("target_n_queries", ctypes.c_uint32),
        ("reserved", ctypes.c_int32 * 2),
    ]


class sng_frame_result(ctypes.Structure):
    _fields_ = [
        ("d_final_rgba", ctypes.c_void_p),
        ("d_final_depth", ctypes.c_void_p),
        ("d_nerf_rgba", ctypes.c_void_p),
        ("d_nerf_depth", ctypes.c_void_p),
        ("d_nerf_positions", ctypes.c_void_p),
        ("d_nerf_normals", ctypes.c_void_p),
        ("d_syn_rgba", ctypes.c_void_p),
        ("d_syn_depth", ctypes.c_void_p),
        ("n_iterations", ctypes.c_uint32),
        ("n_hit", ctypes.c_uint32),
        ("n_samples", ctypes.c_uint64),
        ("n_reference_slots", ctypes.c_uint64),
        ("ms_frame", ctypes.c_float),
        ("ms_raytrace", ctypes.c_float),
        ("ms_nerf", ctypes.c_float),
        ("ms_shadow", ctypes.c_float),
        ("ms_overlay", ctypes.c_float),
        ("ms_network", ctypes.c_float),
        ("network_launches", ctypes.c_uint32),
        ("alive_per_iter", ctypes.c_uint32 * 64),
        ("steps_per_iter", ctypes.c_uint32 * 64),
        ("samples_per_iter", ctypes.c_uint32 * 64),
        ("fused_from_iter", ctypes.c_uint32),
        ("n_samples_network", ctypes.c_uint64),
        ("ms_fused_tail", ctypes.c_float),
        ("n_samples_reused", ctypes.c_uint64),
        ("onestep_from_iter", ctypes.c_uint32),
        ("onestep_iterations", ctypes.c_uint32),
        ("ms_onestep", ctypes.c_float),
        ("onestep_field_evals", ctypes.c_uint32),
        ("spec_rounds", ctypes.c_uint32),
        ("spec_evals", ctypes.c_uint32),
        ("spec_exec", ctypes.c_uint32),
        ("msr_rounds", ctypes.c_uint32),
        ("msr_evals", ctypes.c_uint32),
        ("msr_exec", ctypes.c_uint32),
        ("sched_reductions", ctypes.c_uint32),
        ("n_launch_rec", ctypes.c_uint32),
        ("ms_network_launch", ctypes.c_float * 16),
        ("samples_network_launch", ctypes.c_uint32 * 16),
    ]


class sng_lens(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("params", ctypes.c_float * 7)]


class sng_light(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 3), ("intensity", ctypes.c_float), ("size", ctypes.c_float), ("type", ctypes.c_int32)]


class sng_material(ctypes.Structure):
    _fields_ = [
        ("ka", ctypes.c_float * 3),
        ("kd", ctypes.c_float * 3),
        ("ks", ctypes.c_float * 3),
        ("n", ctypes.c_float),
        ("rg", ctypes.c_float),
        ("spec_angle", ctypes.c_float),
        ("type", ctypes.c_int32),
    ]


class sng_object_info(ctypes.Structure):
    _fields_ = [
        ("n_nodes", ctypes.c_uint32),
        ("n_tris", ctypes.c_uint32),
        ("rot", ctypes.c_float * 9),
        ("pos", ctypes.c_float * 3),
        ("scale", ctypes.c_float),
        ("mat_id", ctypes.c_int32),
    ]


P = ctypes.c_void_p
U32 = ctypes.c_uint32
U64 = ctypes.c_uint64
I32 = ctypes.c_int32
F32 = ctypes.c_float
FP = ctypes.POINTER(ctypes.c_float)
U16P = ctypes.POINTER(ctypes.c_uint16)
U32P = ctypes.POINTER(ctypes.c_uint32)

class sng_train_stats(ctypes.Structure):
    _fields_ = [
        ("step", ctypes.c_uint32),
        ("loss", ctypes.c_float),
        ("rays_per_batch", ctypes.c_uint32),
        ("measured_batch", ctypes.c_uint32),
        ("measured_batch_before_compaction", ctypes.c_uint32),
        ("ms", ctypes.c_float),
        ("ms_generate", ctypes.c_float),
        ("ms_network", ctypes.c_float),
        ("ms_loss", ctypes.c_float),
        ("ms_grad_clear", ctypes.c_float),
        ("ms_field", ctypes.c_float),
        ("ms_dw", ctypes.c_float),
        ("ms_optimizer", ctypes.c_float),
        ("timed_steps", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 2),
    ]


SNG_COMM_ID_BYTES = 128
# int (*sng_sched_reduce_fn)(uint32_t* values, uint32_t n, void* user)
SCHED_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_void_p)

# name -> (restype, argtypes); every symbol declared in include/sng.h
SIGNATURES = {
    "sng_last_error": (ctypes.c_char_p, []),
    "sng_abi_version": (ctypes.c_int, []),
    "sng_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "sng_ctx_create": (ctypes.c_int, [ctypes.POINTER(sng_ctx_desc), ctypes.POINTER(P)]),
    "sng_ctx_destroy": (ctypes.c_int, [P]),
    "sng_load_snapshot": (ctypes.c_int, [P, ctypes.c_char_p]),
    "sng_save_snapshot": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32]),
    "sng_rt_counters": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint64)]),
    "sng_gather_rgba8": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int32), P, P]),
    "sng_comm_allreduce_u32": (ctypes.c_int, [P, P, ctypes.c_uint64, P]),
    "sng_frame_buffer": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "sng_snapshot_probe": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(sng_nerf_config), ctypes.POINTER(U64), ctypes.POINTER(U64), U16P, U64,
                                          U16P, U64]),
    "sng_set_nerf_model": (ctypes.c_int, [P, ctypes.POINTER(sng_nerf_config), U16P, U64]),
    "sng_nerf_param_count": (U64, [ctypes.POINTER(sng_nerf_config)]),
    "sng_set_density_grid": (ctypes.c_int, [P, U16P, U64]),
    "sng_get_bitfield": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint8), U64]),
    "sng_get_density_mean": (ctypes.c_int, [P, FP]),
    "sng_nerf_inference": (ctypes.c_int, [P, P, U32, U32, P, I32, P]),
    "sng_hashgrid_encode": (ctypes.c_int, [P, P, U32, U32, P, P]),
    "sng_sh_encode": (ctypes.c_int, [P, P, U32, U32, U32, P, P]),
    "sng_load_virtual_scene": (ctypes.c_int, [P, ctypes.c_char_p]),
    "sng_clear_virtual_scene": (ctypes.c_int, [P]),
    "sng_set_param": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.c_double]),
    "sng_get_param": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    "sng_get_scene_counts": (ctypes.c_int, [P, U32P, U32P, U32P]),
    "sng_get_object": (ctypes.c_int, [P, U32, ctypes.POINTER(sng_object_info)]),
    "sng_get_object_bvh": (ctypes.c_int, [P, U32, FP, FP]),
    "sng_get_light": (ctypes.c_int, [P, U32, ctypes.POINTER(sng_light)]),
    "sng_get_material": (ctypes.c_int, [P, U32, ctypes.POINTER(sng_material)]),
    "sng_set_camera_view": (ctypes.c_int, [P, FP, FP, F32]),
    "sng_set_camera_matrix": (ctypes.c_int, [P, FP]),
    "sng_get_camera_matrix": (ctypes.c_int, [P, FP]),
    "sng_set_motion_blur": (ctypes.c_int, [P, FP, FP]),
    "sng_set_fov": (ctypes.c_int, [P, F32]),
    "sng_get_focal_length": (ctypes.c_int, [P, ctypes.c_int, FP]),
    "sng_set_window": (ctypes.c_int, [P, I32, I32]),
    "sng_get_resolution": (ctypes.c_int, [P, ctypes.POINTER(sng_resolution_info)]),
    "sng_render_frame": (ctypes.c_int, [P, ctypes.POINTER(sng_frame_params), ctypes.POINTER(sng_frame_result)]),
    "sng_render_nerf_ngp": (ctypes.c_int, [P, ctypes.POINTER(sng_frame_params), ctypes.POINTER(sng_frame_result)]),
    "sng_display_frame": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint8), U64]),
    "sng_save_image": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.POINTER(I32)]),
    "sng_image_write_png": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint8), I32, I32, I32]),
    "sng_animation_probe": (ctypes.c_int, [ctypes.c_char_p, U32, I32, ctypes.c_float, FP, FP, U32, FP, U32, ctypes.POINTER(U32),
                                           ctypes.POINTER(U32)]),
    "sng_image_load_png": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint8), U64, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
    "sng_train_set_dataset": (ctypes.c_int, [P, U32, U32, U32, ctypes.POINTER(ctypes.c_uint8), FP, FP, FP]),
    "sng_train_set_lens": (ctypes.c_int, [P, ctypes.POINTER(sng_lens), U32]),
    "sng_set_render_lens": (ctypes.c_int, [P, ctypes.POINTER(sng_lens)]),
    "sng_get_render_lens": (ctypes.c_int, [P, ctypes.POINTER(sng_lens)]),
    "sng_set_camera_to_training_view": (ctypes.c_int, [P, ctypes.c_int32]),
    "sng_train_reset": (ctypes.c_int, [P, U64]),
    "sng_train": (ctypes.c_int, [P, U32, ctypes.POINTER(sng_train_stats)]),
    "sng_train_export": (ctypes.c_int, [P, U16P, U64, U16P, U64]),
    "sng_train_debug": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_char_p, P, U64, ctypes.POINTER(U64)]),
    "sng_comm_unique_id": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint8)]),
    "sng_set_comm": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int]),
    "sng_set_sched_reducer": (ctypes.c_int, [P, P, P]),
    "sng_set_sched_replay": (ctypes.c_int, [P, U32P, U64]),
    "sng_synchronize": (ctypes.c_int, [P]),
    "sng_copy_to_host": (ctypes.c_int, [P, P, P, U64]),
    "sng_copy_device": (ctypes.c_int, [P, P, P, U64, P]),
    "sng_final_rgba8": (ctypes.c_int, [P, ctypes.c_int32, ctypes.c_int32, P, P]),
    "sng_get_rng_states": (ctypes.c_int, [P, ctypes.c_int, U32P, U64]),
    "sng_set_rng_states": (ctypes.c_int, [P, ctypes.c_int, U32P, U64]),
    "sng_bvh_build": (ctypes.c_int, [FP, U32, U32, FP, U32, U32P]),
}

_lib = None


ABI_VERSION = 4   # SNG_ABI_VERSION of include/sng.h


def load():
    """Load libsng_hip.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libsng_hip.so not built ({LIB_PATH}); run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sng_abi_version() != ABI_VERSION:   # the struct mirrors below follow include/sng.h of this version
        raise ImportError(f"libsng_hip.so ABI {lib.sng_abi_version()} != {ABI_VERSION}; rebuild it")
    _lib = lib
    return lib


def check(status):
    if status != SNG_OK:
        msg = load().sng_last_error().decode(errors="replace")
        raise SngError(f"sng error {status}: {msg}")
    return status
