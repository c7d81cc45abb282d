// host_params.cpp -- the engine parameters (sng_set_param / sng_get_param keys): each with the reference member it
// stands for, or what it switches in this implementation.
#include "host.h"

namespace sng_host {

const std::map<std::string, double>& default_params() {
    static const std::map<std::string, double> d = {
        {"res_factor", 64},                     // Testbed::m_fixed_res_factor (testbed.h:656)
        {"vo_scale", 4},                        // Engine::m_relative_vo_scale (engine.cuh:113)
        {"exposure", 0.0},                      // Testbed::m_exposure
        {"tonemap_curve", 0},                   // Testbed::m_tonemap_curve (engine.cu:406): 0 Identity, 1 ACES, 2 Hable, 3 Reinhard
        {"rt_buffer_type", 0},                  // RayTracer::m_buffer_to_show (raytracer.cuh:20,179): 0 Final, 1 NextOrigin, 2 SrcOrigin,
                                                //   3 NextDirection, 4 SrcDirection, 5 Normal, 6 Depth, 7 NerfShadow
        {"path_trace_depth", 2},                // RayTracer::m_ray_iters (raytracer.cuh:160)
        {"light_samples", 2},                   // RayTracer::m_samples
        {"syn_shadow_samples", 4},              // RayTracer::m_shadow_iters
        {"syn_shadow_intensity", 1.0},          // RayTracer::m_syn_shadow_factor
        {"attenuation", 1.0},                   // RayTracer::m_attenuation_coeff (unused by raytrace)
        {"lens_size", 0.009},                   // RayTracer::m_lens_angle_constant
        {"depth_offset", 0.1},                  // RayTracer::m_depth_offset (overlay z-test)
        {"n_steps", 8},                         // RayTracer::m_n_steps (NeRF shadow steps on meshes)
        {"nerf_shadow_samples", 1},             // Testbed::sng_position_kernel_size (testbed.h:686)
        {"nerf_shadow_intensity", 2.0},         // Engine::m_nerf_shadow_intensity (engine.cuh:117)
        {"nerf_ao_intensity", 2.0},             // Engine::m_nerf_ao_intensity
        {"nerf_on_nerf_shadow_threshold", 0.3}, // Engine::m_nerf_self_shadow_threshold
        {"shadow_on_nerf", 1},                  // Engine::m_view_syn_shadow
        {"shadow_on_virtual_obj", 1},           // RayTracer::m_view_nerf_shadow
        {"show_virtual_obj", 1},                // RayTracer::m_show_virtual_obj
        {"show_nerf", 1},                       // Engine::m_show_nerf
        {"min_transmittance", 0.01},            // render_min_transmittance (testbed.h:867)
        {"srgb", 1},                            // EColorSpace::SRGB passed to overlay (engine.cu:406)
        {"smooth_threshold", 1.0},              // sng_position_kernel_threshold (unused by the path)
        {"max_shadow_variance", 0.0},           // sng_shadow_depth_variance (unused by the path)
        {"concurrent_streams", 1},              // 1: raytracer and NeRF streams overlap (engine.cu:386-405 run them back to back)
        {"rt_start_chunk", 0},                  // concurrent mode: 0 the raytracer starts at frame start beside init_rays; k > 0 its path
                                                //   kernel waits for the head's network launch (the first speculative round's, or the
                                                //   wavefront's of chunk k); -1: 1 for bands of >= 60 % of the rows, else 0.  C3 A/B
                                                //   (round 5, 4 alternating pairs): 0 -> 295-298 frames/s, 1 -> 271-272 (the path kernel,
                                                //   the frame's critical path, idles ~0.3 ms behind init_rays + generate + network)
        {"rt_reserved_cus", 32},                // concurrent mode: CUs (4 per XCD) the persistent raytracer grids leave to the NeRF stream
        {"linear_marcher", 1},                  // exact unit-cube fast path of the occupancy march
        {"occ_lin_all", 1},                     // cascaded marchers read every cascade's occupancy from x-fastest rows (same bits, no Morton code)
        {"fast_slab", 1},                       // exact reciprocal-multiply BVH box tests
        {"rt_wavefront", 1},                    // deferred shadow-ray queues for the path tracer
        {"bvh_wide", 1},                        // traversal layout with both child boxes per record (exact)
        {"bvh_flat", 1},                        // BvhWide walk keeping the nearer child in a register (exact)
        {"rt_tile", 8},                         // path-kernel tile width: 8 (8x8 pixels per wave) or 4 (4x4, shorter chains)
        {"rt_tile_h", 0},                       // path-kernel tile height: 0 = rt_tile; 4 with rt_tile 8: 8x4 (32 lanes per wave)
        {"scene_lds", 1},                       // BVH nodes + triangles staged in LDS per workgroup when they fit
        {"rt_tile_order", 1},                   // visit raytracer tiles in descending previous-frame cost
        {"rt_prio_frac", 0.1},                  // the costliest fraction of the path tiles (last frame's order) at wave priority 3
        {"rt_prio2_frac", 0.25},                // ... the tiles up to this fraction of the order at priority 2
        {"rt_first", 1},                        // concurrent frames: init_rays waits (device-side, bounded) for the path kernel's first workgroup
        {"rt_first_timeout_us", 100},           // ... at most this long
        {"rt_fused_shadow", 1},                 // banded frames: the path kernel's idle waves trace the shadow rays (mesh.hip fq_consume)
        {"rt_fused_tiles_per_wave", 1},         // ... when the band has at most this many path tiles per wave (a full queue is traced in place)
        {"rt_fused_shadow_used", 0},            // (output) 1 when the last frame's path kernel traced its shadow rays itself
        {"rt_spread", 1},                       // the path kernel's first tiles dealt across all CUs (costliest one per CU / SIMD)
        {"rt_rng", 0},                          // 1: a measurement mode, NOT the reference's RNG order -- each (pixel, sample) its own XORWOW
                                                //   subsequence, a pixel's samples traced on adjacent lanes (raytrace_sp_kernel); same
                                                //   expectation, other noise (tests/test_gpu_rt_rng.py); for the band-scaling question
        {"nerf_gbuffer", 0},                    // 1: NeRF normals every frame (otherwise only when shadow_on_nerf needs them)
        {"rt_plist", 1},                        // per-pixel hit-record lists for the colour replay (rt_accumulate_kernel)
        {"glow_mode", 0},                       // Testbed::Nerf::glow_mode (testbed.h:871): bits 1 green grid, 2 cut line, 4 mask to alpha,
                                                // 8 radial, 16 grid mode -- instant-NGP path only (testbed_nerf.cu:638-734)
        {"glow_y_cutoff", 0},                   // Testbed::Nerf::glow_y_cutoff (testbed.h:870)
        {"render_mode", 1},                     // ERenderMode of the instant-NGP path (sng_render_nerf_ngp): Shade
        {"visualized_layer", 0},                // Testbed::m_visualized_layer (testbed.h:1024)
        {"visualized_dimension", -1},           // Testbed::m_visualized_dimension (testbed.h:1023); > -1 selects EncodingVis (testbed_nerf.cu:2491)
        {"train_grid_est", 0},                  // > 0: the per-ray training kernels' grid sized for this many rays (tests of their grid-stride loops)
        {"train_overlap", 1},                   // the next step's generate on a second stream beside this step's gradients / optimizer
        {"train_overlap_tail", 0},              // tests: sng_train also generates the next step ahead, for the parity hook
        {"train_grid_morton", 1},               // density-grid update: the uniform samples in the Morton order of their cells (same samples, same grid)
        {"train_gen_bricks", 0},                // training generator's occupancy: 0 the linear words (measured fastest, tools/train_ab.py), 1 the OccBrick blob (LDS when it fits, else global)
        {"train_grid_grad_f16", 1},             // hash-grid gradients in fp16 with packed atomics, tcnn's grad_t (__half2 atomicAdd); 0: f32
        {"train_grid_density_only", 1},         // density-grid update: the density MLP alone (NerfNetwork::density), not the full network
        {"train_dw_pipe", 1},                   // dW kernel: the next tile's operands in flight during the current tile's MFMAs (0: load, then multiply)
        {"train_dw_blocks_per_cu", 2},          // dW kernel: workgroups per CU (tools/train_ab.py)
        {"train_gen_lanes", 8},                 // lanes per ray of the training generator's speculative march (8 or 16; 1: one lane per ray; tools/train_ab.py)
        {"train_kernel_times", 0},              // 1: sng_train times the stages of every step with HIP events (sng_train_stats.ms_*)
        {"render_with_lens_distortion", 0},     // Testbed::Nerf::render_with_lens_distortion (testbed_nerf.cu:2504): NeRF rays through
                                                //   render_lens (sng_set_render_lens; the snapshot dataset's first lens)
        {"depth_scale", 1.0},                   // 1 / dataset.scale (testbed_nerf.cu:2748)
        {"rt_queue_gb", 48},                    // device-memory budget for the deferred-shadow queues
        {"train_batch", 262144},                // m_training_batch_size (testbed.h:1103)
        {"train_random_bg", 1},                 // m_nerf.training.random_bg_color (testbed.h:790)
        {"train_debug", 0},                     // parity hook: generate writes per-ray step counts (sng_train_debug)
        {"nerf_fused", 1},                      // ray-local fused NeRF kernel for the tail iterations (fused.hip)
        {"nerf_fused_after", 0},                // ... after this many whole-GPU wavefront iterations (0: the speculative tail
                                                //   from the first iteration, queued ahead of its device check; C2 1311 -> 1483
                                                //   frames/s against 1, C3 unchanged)
        {"nerf_spec_rounds", 2},                // speculative tail rounds before the fused kernel finishes the stragglers (nerf.hip)
        {"nerf_spec_adapt", 1},                 // ... (hybrid frames, NeRF tail beside the raytracer) one round fewer while the
                                                //   last frame's final round evaluated fewer than
        {"nerf_spec_min_samples", 8192},        //   this many samples (a whole-GPU launch for them costs more than the fused
                                                //   kernel does), one more when the rays that kernel takes over would fill
                                                //   one twice over (exact either way)
        {"nerf_spec_budget", 16777216},         // samples one round may generate (K = clamp(budget / (8 n_alive), 1, kmax)); the
                                                //   sample buffers are sized for it (16.8 M x 60 B ~ 1 GB of the 288 GB)
        {"nerf_spec_hint", 1},                  // a ray looks ahead as far as its pixel's ray lived last frame (exact; 0: opacity policy)
        {"nerf_spec_hint_any_view", 0},         // 1: read the hints whatever view wrote them (tests: exact for any hint)
        {"nerf_spec_kmax", 16},                 // iterations one round marches ahead (<= 16)
        {"nerf_spec_k_policy", 1},              // per-ray look-ahead from the ray's opacity in all rounds but the last (exact)
        {"nerf_spec_prepare", 1},               // sample-parallel activations before the spec compositor (exact; 0: in the chain)
        {"occ_lds_kb", 64},                     // LDS budget for the occupancy bricks in the linear marchers (0: global loads)
        {"load_optimizer_state", 1},            // sng_load_snapshot restores a snapshot's optimizer state (0: inference model only)
        {"optimizer_state_loaded", -1},         // set by sng_load_snapshot: 1 restored, 0 skipped / malformed, -1 none in the file
        {"nerf_fused_lanes", 64},               // rays per wave in the fused kernel
        {"nerf_fused_blocks", -1},              // workgroup cap of the fused kernel (0: 2 per CU; -1: 2 per reserved CU when concurrent)
        {"nerf_gen_blocks", -1},                 // generate grid (256-thread units): 0 = min(rays, 8 per CU); -1 = all rays in one trip
        {"rt_shadow_all_cus", 1},               // shadow-ray kernel on every CU: the NeRF tail has mostly finished by then (C3 +2 %; 0: the path kernel grid)
        {"rt_count", 0},                        // count BVH queries / box / triangle tests of the deferred raytracer (sng_rt_counters); 2: wave iterations
        {"nerf_msr", 1},                        // multi-step speculative rounds while n_steps is 2..7 (nerf.hip msr_*; exact)
        {"nerf_msr_budget", 16777216},          // samples one such round may generate (K = clamp(budget / (S n_alive), 1, kmax))
        {"nerf_msr_kmax", 16},                  // iterations one such round marches ahead (<= 16)
        {"nerf_msr_span", -1},                  // rounds follow the last frame's schedule across step changes (1), not (0), -1: on banded frames
        {"march_log", 0},                       // diagnostics: log {alive, steps, samples} of every iteration (sng_frame_buffer "march_log")
        {"nerf_onestep", 1},                    // trace_alt's one-step regime (n_alive > target / 2) ray-local and speculative (fused.hip)
        {"nerf_onestep_horizon", 2048},         // iterations one speculative segment of the regime spans
    };
    return d;
}

}  // namespace sng_host
