// host_train.cpp -- online training (BASELINE config 5): Testbed::train_nerf + training_prep_nerf
// (testbed_nerf.cu:3298-3780) on the kernels of train.hip.
#include "host.h"

namespace sng_host {

TrainImages train_images(sng_ctx* c) {
    auto& t = c->tr;
    return {t.pixels.as<uint32_t>(), t.xforms.as<float>(), t.xforms_ray.as<float>(), t.focal.as<float>(), t.pp.as<float>(),
            t.h_lens.empty() ? nullptr : t.lens.as<Lens>(), t.w, t.h, t.n_images};
}

// Testbed::reset_network's training state: fp32 master weights from the current model, zeroed
// optimizer moments, m_rng = pcg32(seed), density_grid_rng = pcg32(m_rng.next_uint()) (testbed.cu:3654-3667)
// a step generated ahead on s_gen (train_overlap_tail) is discarded: wait for its kernels, then the next step generates
// its own samples from the current state
void train_drop_pregen(sng_ctx::Train& t) {
    if (t.pregen) { HIPCHK(hipStreamSynchronize(t.s_gen)); t.pregen = false; }
}

void train_reset(sng_ctx* c, uint64_t seed) {
    if (!c->has_model) throw SngError(SNG_ERR_STATE, "set or load a model before training");
    auto& t = c->tr;
    const uint64_t n = c->n_params;
    t.master.ensure(n * 4); t.grads.ensure(n * 4); t.m1.ensure(n * 4); t.m2.ensure(n * 4); t.steps.ensure(n * 4); t.ema.ensure(n * 4);
    t.p_train.ensure(n * 2); t.p_infer.ensure(n * 2);
    t.wfrag_train.ensure(20 * 512 * 2); t.wfrag_t.ensure(36 * 256 * 2);
    std::vector<uint16_t> h(n);
    HIPCHK(hipMemcpy(h.data(), c->d_params.p, n * 2, hipMemcpyDeviceToHost));
    std::vector<float> f(n);
    for (uint64_t i = 0; i < n; ++i) f[i] = h2f(h[i]);
    HIPCHK(hipMemcpy(t.master.p, f.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.ema.p, f.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_train.p, h.data(), n * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_infer.p, h.data(), n * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(t.m1.p, 0, n * 4)); HIPCHK(hipMemset(t.m2.p, 0, n * 4)); HIPCHK(hipMemset(t.steps.p, 0, n * 4));
    const uint32_t n_cells = GRID_CELLS * (c->max_cascade + 1);
    t.grid.ensure((size_t)n_cells * 4); t.grid_tmp.ensure((size_t)n_cells * 4);
    HIPCHK(hipMemset(t.grid.p, 0, (size_t)n_cells * 4));
    t.rng = Pcg32::seeded(seed);
    t.grid_rng = Pcg32::seeded(t.rng.next_uint());
    t.step = 0; t.grid_ema_step = 0; t.rays_per_batch = 1u << 12; t.measured = 0; t.measured_before = 0;
    t.sched.ensure(sizeof(TrainSched));
    t.sched_dirty = true;
    train_drop_pregen(t);   // a step generated ahead belongs to the old run
    t.target = (uint32_t)c->p("train_batch");
    const uint32_t target = t.target, max_samples = target * 16;
    t.ctrl.ensure(sizeof(TrainCtrl));
    const size_t max_rays = 1u << 18;   // rays_per_batch is capped at 2^18 (update_after_training)
    t.ray_indices.ensure(max_rays * 4); t.rays.ensure(max_rays * 32); t.numsteps.ensure(max_rays * 8);
    t.coords.ensure((size_t)max_samples * 28); t.mlp_out.ensure((size_t)max_samples * 8);
    t.coords_c.ensure((size_t)target * 28); t.dloss.ensure((size_t)target * 8); t.loss.ensure(max_rays * 4);
    t.acts.ensure((size_t)((target + 15) / 16) * TRAIN_FEATS * 16 * 2);
    t.partial.ensure((size_t)max_samples * 16); t.rayrec.ensure(max_rays * 48);
    t.cnt_i.ensure(max_rays * 4); t.cbase_i.ensure(max_rays * 4);
    t.tscr.ensure(max_rays * NERF_STEPS * 4);   // strided by the device's ray count, which the host does not wait for
    if (!t.h_sched) HIPCHK(hipHostMalloc((void**)&t.h_sched, 2 * sizeof(TrainSched), hipHostMallocDefault));
    for (hipEvent_t& e : t.sched_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the bitfield the training marcher reads (density grid -> bitfield after every update)
    c->d_grid_f32.ensure((size_t)n_cells * 4);
    c->d_partial.ensure(1024 * sizeof(double));
    c->d_mean.ensure(sizeof(float));
    c->d_bitfield.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);
    c->d_occ_linear.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);   // every cascade (Volume::occ_lin_all)
    t.ready = true;
}

NetworkDev train_net(sng_ctx* c, const DevBuf& params, const DevBuf& wfrag) {
    NetworkDev n = c->net;
    n.wfrag = wfrag.p;
    n.grid = static_cast<uint16_t*>(params.p) + 3072 + 7168;
    return n;
}

// update_density_grid_nerf (testbed_nerf.cu:3121-3210) + update_density_grid_mean_and_bitfield
void train_density_update(sng_ctx* c, hipStream_t s) {
    auto& t = c->tr;
    const uint32_t n_casc = c->max_cascade + 1, n_cells = GRID_CELLS * n_casc;
    if (t.step == 0) {
        t.grid_ema_step = 0;
        launch_train_mark_untrained(n_cells, t.grid.as<float>(), train_images(c), 1, s);
    }
    const uint32_t n_uni = t.step < 256 ? n_cells : n_cells / 4, n_non = t.step < 256 ? 0 : n_cells / 4;
    const uint32_t n_tot = n_uni + n_non;
    t.grid_coords.ensure((size_t)n_tot * 28); t.grid_idx.ensure((size_t)n_tot * 4); t.grid_out.ensure((size_t)n_tot * 8);
    HIPCHK(hipMemsetAsync(t.grid_tmp.p, 0, (size_t)n_cells * 4, s));
    const int morton = c->p("train_grid_morton") != 0.0 ? 1 : 0;
    launch_train_grid_samples(n_uni, t.grid_rng, t.grid_ema_step, c->box, t.grid.as<float>(), t.grid_coords.as<float>(), t.grid_idx.as<uint32_t>(), n_casc, -0.01f,
                              morton, s);
    t.grid_rng.advance();
    launch_train_grid_samples(n_non, t.grid_rng, t.grid_ema_step, c->box, t.grid.as<float>(), t.grid_coords.as<float>() + (size_t)n_uni * 7,
                              t.grid_idx.as<uint32_t>() + n_uni, n_casc, NERF_MIN_OPTICAL_THICKNESS, morton, s);
    t.grid_rng.advance();
    // density of the training parameters (m_nerf_network->density, use_inference_params = false)
    launch_train_pack(t.p_train.as<uint16_t>(), t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s);
    launch_network(train_net(c, t.p_train, t.wfrag_train), t.grid_coords.as<float>(), 7, n_tot, nullptr, t.grid_out.as<uint16_t>(),
                   c->p("train_grid_density_only") != 0.0 ? 2 : 1, 0, s);
    launch_train_grid_splat_ema(n_tot, t.grid_idx.as<uint32_t>(), t.grid_out.as<uint16_t>(), t.grid_tmp.as<float>(), n_cells, 0.95f, t.grid.as<float>(), s);
    ++t.grid_ema_step;
    HIPCHK(hipMemcpyAsync(c->d_grid_f32.p, t.grid.p, (size_t)n_cells * 4, hipMemcpyDeviceToDevice, s));
    launch_bitfield(nullptr, c->max_cascade, c->d_grid_f32.as<float>(), c->d_partial.as<double>(), c->d_mean.as<float>(), c->d_bitfield.as<uint8_t>(),
                    c->d_occ_linear.as<uint32_t>(), s);
    build_occ_brick(c, s);
    c->has_bitfield = true;
}

TrainStepArgs train_args(sng_ctx* c) {
    auto& t = c->tr;
    TrainStepArgs a{};
    a.vol = make_volume(c);
    a.sched = t.sched.as<TrainSched>();
    a.n_rays_grid = std::min(t.n_rays_est + t.n_rays_est / 4, 1u << 18);   // a lagged estimate plus room for its growth
    if (c->p("train_grid_est") > 0.0) a.n_rays_grid = (uint32_t)c->p("train_grid_est");   // tests: force the kernels' grid-stride trips
    a.target_batch = t.target;
    a.random_bg = c->p("train_random_bg") != 0.0 ? 1 : 0;
    a.background = mk(0.0f, 0.0f, 0.0f);
    a.loss_scale = 128.0f;   // default_loss_scale<__half>
    a.near_distance = 0.1f;
    a.debug = c->p("train_debug") != 0.0 ? 1 : 0;
    a.gen_bricks = c->p("train_gen_bricks") != 0.0 ? 1 : 0;
    a.gen_lanes = (int)c->p("train_gen_lanes");
    a.dw_pipe = c->p("train_dw_pipe") != 0.0 ? 1 : 0;
    a.dw_blocks_per_cu = std::max(1, (int)c->p("train_dw_blocks_per_cu"));
    a.grid_grad_f16 = c->p("train_grid_grad_f16") != 0.0 && c->net.F == 4 ? 1 : 0;
    return a;
}

TrainBatch train_batch(sng_ctx* c) {
    auto& t = c->tr;
    return {t.ctrl.as<TrainCtrl>(), t.ray_indices.as<uint32_t>(), t.rays.as<float4>(), t.numsteps.as<uint2>(), t.coords.as<float>(), t.mlp_out.as<uint16_t>(),
            t.coords_c.as<float>(), t.dloss.as<uint16_t>(), t.loss.as<float>(), t.acts.as<uint16_t>(), t.partial.as<float4>(), t.rayrec.as<float4>(),
            t.cnt_i.as<uint32_t>(), t.cbase_i.as<uint32_t>()};
}

// train_nerf_step (3532-3780) up to the gradients; stage > 0 stops early (parity hooks):
// 1 = samples generated, 2 = network outputs, 3 = loss / compaction, 4 = gradients
// ev (train_kernel_times): 8 events bracketing generate | network | loss | gradient clear | field | dW (the optimizer's
// event is recorded by train_steps)
void train_sched_push(sng_ctx* c, hipStream_t s) {
    auto& t = c->tr;
    if (t.sched_dirty) {   // host-set batch sizes (reset, snapshot load): train_args' max_inference from measured_before
        const uint32_t cap = t.target * 16;
        const TrainSched h{t.rays_per_batch,
                           t.measured_before == 0 ? cap : (std::min(t.measured_before, cap) + BATCH_SIZE_GRANULARITY - 1) / BATCH_SIZE_GRANULARITY * BATCH_SIZE_GRANULARITY,
                           t.measured, t.measured_before};
        HIPCHK(hipMemcpyAsync(t.sched.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));   // h is a stack value
        t.n_rays_est = t.rays_per_batch;
        t.sched_dirty = false;
    }
}

// the step's first stage: the per-ray buffers cleared, the samples generated (rng: the step's stream)
void train_generate_stage(sng_ctx* c, const Pcg32& rng, hipStream_t s) {
    auto& t = c->tr;
    const TrainStepArgs a = train_args(c);
    const TrainBatch b = train_batch(c);
    launch_train_clear(a, b, s);   // also zeroes the batch counters (TrainCtrl)
    launch_train_generate(a, train_images(c), b, rng, t.tscr.as<float>(), s);
}

// generated: the step's samples were queued ahead on the generator stream (train_steps); ev_loss: recorded after the
// loss stage (the next step's generate may start from there)
void train_forward_backward(sng_ctx* c, int stage, hipStream_t s, hipEvent_t* ev, bool generated, hipEvent_t ev_loss) {
    auto& t = c->tr;
    train_sched_push(c, s);
    const TrainStepArgs a = train_args(c);
    const TrainBatch b = train_batch(c);
    const TrainImages im = train_images(c);
    auto mark = [&](int k) { if (ev) HIPCHK(hipEventRecord(ev[k], s)); };
    if (!generated) {
        launch_train_clear(a, b, s);   // also zeroes the batch counters (TrainCtrl)
        mark(0);
        launch_train_generate(a, im, b, t.rng, t.tscr.as<float>(), s);
        mark(1);
    }
    if (stage == 1) return;
    // inference forward of every sample with the training params
    // with the network's count = min(numsteps_counter, max_samples): the generator drops rays beyond max_samples
    launch_train_pack(t.p_train.as<uint16_t>(), t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s, &b.ctrl->numsteps_counter, a.sched,
                      t.ctrl.as<uint32_t>() + 3);
    const NetworkDev net = train_net(c, t.p_train, t.wfrag_train);
    launch_network(net, b.coords, 7, 0, t.ctrl.as<uint32_t>() + 3, b.mlp_out, 1, (t.target * 16 + 15) / 16, s);
    mark(2);
    if (stage == 2) return;
    launch_train_loss(a, im, b, t.rng, c->d_mean.as<float>(), stage == 0 ? t.sched.as<TrainSched>() : nullptr, s);
    if (ev_loss) HIPCHK(hipEventRecord(ev_loss, s));
    mark(3);
    if (stage == 3) return;
    const uint64_t n_mlp = 3072 + 7168;
    t.grads_h_used = a.grid_grad_f16 != 0;
    if (t.grads_h_used) {   // f32 MLP gradients + fp16 grid gradients (tcnn's grad_t)
        t.grads_h.ensure((c->n_params - n_mlp) * 2);
        HIPCHK(hipMemsetAsync(t.grads.p, 0, n_mlp * 4, s));
        HIPCHK(hipMemsetAsync(t.grads_h.p, 0, (c->n_params - n_mlp) * 2, s));
    } else {
        HIPCHK(hipMemsetAsync(t.grads.p, 0, c->n_params * 4, s));
    }
    mark(4);
    float* g = t.grads.as<float>();
    launch_train_field(a, b, net, t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), static_cast<uint16_t*>(net.grid), g + n_mlp,
                       t.grads_h_used ? t.grads_h.as<uint16_t>() : nullptr, s);
    mark(5);
    launch_train_dw(a, b.acts, g, (uint32_t)c->n_cus, s);
    mark(6);
}

void train_steps(sng_ctx* c, uint32_t n_steps, sng_train_stats* out) {
    if (!c->tr.ready) train_reset(c, 1337);
    auto& t = c->tr;
    if (t.n_images == 0) throw SngError(SNG_ERR_STATE, "no training images (sng_train_set_dataset)");
    hipStream_t s = c->s_nerf;
    HIPCHK(hipEventRecord(c->ev_start, s));
    double loss_acc = 0.0;
    // per-stage device times (param train_kernel_times): generate, network, loss, gradient clear, field, dW, optimizer
    const bool timed = c->p("train_kernel_times") != 0.0;
    while (timed && c->train_events.size() < 8) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); c->train_events.push_back(e); }
    double stage_ms[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t timed_steps = 0;
    const bool overlap = !timed && c->p("train_overlap") != 0.0;
    if (overlap && !t.s_gen) {
        HIPCHK(hipStreamCreateWithFlags(&t.s_gen, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&t.ev_gen, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&t.ev_loss, hipEventDisableTiming));
    }
    // a step generated ahead (train_overlap_tail) is used as is, except under per-stage timing: its generate stage would
    // have no events, so it is generated again in the timed step (the same samples: same rng, grid and batch sizes)
    if (timed) train_drop_pregen(t);
    bool generated = t.pregen;
    t.pregen = false;
    train_sched_push(c, s);
    for (uint32_t k = 0; k < n_steps; ++k) {
        // Testbed::train: training_prep_nerf every clamp(step / 16, 1, 16) steps (testbed.cu:4081-4091)
        const uint32_t skip = std::min(16u, std::max(1u, t.step / 16u));
        if (t.step % skip == 0) train_density_update(c, s);   // never on a step generated ahead (below)
        if (generated) HIPCHK(hipStreamWaitEvent(s, t.ev_gen, 0));
        train_forward_backward(c, 0, s, timed ? c->train_events.data() : nullptr, generated, overlap ? t.ev_loss : nullptr);
        generated = false;
        // the next step's samples depend on this step's batch sizes (formed in the loss stage) and on the occupancy
        // grid, not on the parameters: unless a density-grid update comes first, they are generated on a second stream
        // while this step's gradients and optimizer run (train_overlap; not with per-stage timing)
        if (overlap && k + 1 < n_steps) {
            const uint32_t ns = t.step + 1, skip_n = std::min(16u, std::max(1u, ns / 16u));
            if (ns % skip_n != 0) {
                HIPCHK(hipStreamWaitEvent(t.s_gen, t.ev_loss, 0));
                Pcg32 r = t.rng;
                r.advance();
                train_generate_stage(c, r, t.s_gen);
                HIPCHK(hipEventRecord(t.ev_gen, t.s_gen));
                generated = true;
            }
        }
        // optimizer_step: Ema(ExponentialDecay(Adam)) (base.json)
        AdamArgs o{};
        const uint32_t decays = t.step >= 20000 ? (t.step - 20000) / 10000 + 1 : 0;
        o.lr = 1e-2f * std::pow(0.33f, (float)decays);
        o.beta1 = 0.9f; o.beta2 = 0.99f; o.epsilon = 1e-15f; o.l2_reg = 1e-6f; o.loss_scale = 128.0f; o.ema_decay = 0.95f; o.ema_step = t.step;
        o.deb_old = 1.0f - std::pow(o.ema_decay, (float)o.ema_step);
        o.deb_new = 1.0f - std::pow(o.ema_decay, (float)(o.ema_step + 1));
        // per-parameter step counts reach at most t.step + 1 after this update (a larger one forms the factor itself)
        if (t.adam_corr_n < t.step + 1) {
            const uint32_t need = t.step + 1;
            if (t.adam_corr.bytes < (size_t)(need + 1) * 4) {
                t.adam_corr.ensure(((size_t)need + 4096) / 4096 * 4096 * 4);
                t.adam_corr_n = 0;
            }
            // the table's whole capacity at once (one small launch per 4096 steps instead of one per step)
            const uint32_t to = (uint32_t)(t.adam_corr.bytes / 4) - 1;
            launch_train_adam_corr(t.adam_corr.as<float>(), t.adam_corr_n + 1, to, o.beta1, o.beta2, s);
            t.adam_corr_n = to;
        }
        o.corr = t.adam_corr.as<float>();
        o.corr_n = t.adam_corr_n;
        o.grads_h = t.grads_h_used ? t.grads_h.as<uint16_t>() : nullptr;
        launch_train_adam(o, c->n_params, 3072 + 7168, t.master.as<float>(), t.grads.as<float>(), t.m1.as<float>(), t.m2.as<float>(), t.steps.as<uint32_t>(),
                          t.ema.as<float>(), t.p_train.as<uint16_t>(), t.p_infer.as<uint16_t>(), s);
        if (timed) HIPCHK(hipEventRecord(c->train_events[7], s));
        t.rng.advance();
        ++t.step;
        // NerfCounters::update_after_training (3272-3296) ran on the device at the end of the loss stage (train_rollover_kernel):
        // the next step reads its batch sizes from there, so the host queues the steps without waiting for each (the
        // reference syncs on a readback every step)
        // the grid-size estimate follows the device's ray count through the readback slots (correctness never depends
        // on it: the kernels loop over the device count)
        if (t.step % 8 == 0) {
            const uint32_t q = t.sched_slot;
            if (t.sched_pending[q]) {   // issued 16 steps ago: waits only while the host is further ahead than that
                HIPCHK(hipEventSynchronize(t.sched_ev[q]));
                t.n_rays_est = std::max(t.h_sched[q].n_rays, 256u);
            }
            HIPCHK(hipMemcpyAsync(&t.h_sched[q], t.sched.p, sizeof(TrainSched), hipMemcpyDeviceToHost, s));
            HIPCHK(hipEventRecord(t.sched_ev[q], s));
            t.sched_pending[q] = true;
            t.sched_slot ^= 1u;
        }
        if (timed) {   // per-stage times need the step's events: one wait per step in this mode only
            HIPCHK(hipStreamSynchronize(s));
            for (int q = 0; q < 7; ++q) {
                float ms = 0.0f;
                HIPCHK(hipEventElapsedTime(&ms, c->train_events[q], c->train_events[q + 1]));
                stage_ms[q] += ms;
            }
            ++timed_steps;
        }
    }
    HIPCHK(hipEventRecord(c->ev_end, s));
    // inference params (EMA) -> the render path's weights and grid
    launch_train_pack(t.p_infer.as<uint16_t>(), c->d_wfrag.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s);
    HIPCHK(hipMemcpyAsync(c->d_grid.p, static_cast<uint16_t*>(t.p_infer.p) + 3072 + 7168, (c->n_params - 3072 - 7168) * 2, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_params.p, t.p_infer.p, c->n_params * 2, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    if (n_steps) {   // the device's batch sizes and the last step's counters back to the host
        TrainSched h{};
        TrainCtrl hc{};
        HIPCHK(hipMemcpy(&h, t.sched.p, sizeof(h), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&hc, t.ctrl.p, sizeof(hc), hipMemcpyDeviceToHost));
        t.rays_per_batch = h.n_rays; t.measured = h.measured; t.measured_before = h.measured_before;
        t.n_rays_est = h.n_rays;
        t.sched_pending[0] = t.sched_pending[1] = false;
        if (out) {
            std::vector<float> l(std::max<uint32_t>(1, hc.ray_counter));
            const uint32_t nr = std::min<uint32_t>(hc.ray_counter, (uint32_t)(t.loss.bytes / 4));
            if (nr) HIPCHK(hipMemcpy(l.data(), t.loss.p, nr * 4, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < nr; ++i) loss_acc += l[i];
            t.last_loss = (float)(loss_acc * (double)t.measured / (double)t.target);
        }
    }
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->step = t.step;
        out->loss = t.last_loss;
        out->rays_per_batch = t.rays_per_batch;
        out->measured_batch = t.measured;
        out->measured_batch_before_compaction = t.measured_before;
        HIPCHK(hipEventElapsedTime(&out->ms, c->ev_start, c->ev_end));
        out->timed_steps = timed_steps;
        float* dst[7] = {&out->ms_generate, &out->ms_network, &out->ms_loss, &out->ms_grad_clear, &out->ms_field, &out->ms_dw, &out->ms_optimizer};
        for (int q = 0; q < 7; ++q) *dst[q] = timed_steps ? (float)(stage_ms[q] / timed_steps) : 0.0f;
    }
    // tests (train_overlap_tail): the next step generated ahead as in the loop, for the parity hook to check; queued
    // after the counters above were read back (its generate stage clears the step's control words and losses)
    if (overlap && n_steps && c->p("train_overlap_tail") != 0.0) {
        const uint32_t skip_n = std::min(16u, std::max(1u, t.step / 16u));
        if (t.step % skip_n != 0) {
            HIPCHK(hipStreamWaitEvent(t.s_gen, t.ev_loss, 0));
            train_generate_stage(c, t.rng, t.s_gen);   // t.rng is the next step's stream already
            HIPCHK(hipEventRecord(t.ev_gen, t.s_gen));
            HIPCHK(hipStreamWaitEvent(s, t.ev_gen, 0));
            t.pregen = true;
        }
    }
}

}  // namespace sng_host
