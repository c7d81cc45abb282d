// sng-render -- headless replacement for the reference's instant-ngp executable on the render path
// (main.cu:30-229): the same --snapshot / --virtual / --frag / --width / --height /
// --sshadows / --nshadows flags (main.cu:93-126), so scripts/render/profiling.sh runs against this
// library by swapping EXEC, plus the headless --frames / --out / --gpus.
//
// One process per GPU: with --gpus N the launcher forks N ranks before anything touches the GPU; rank 0
// makes the RCCL unique id and hands it to the others through pipes.  Each rank renders one row band
// of every frame (sng_render_frame with row_begin/row_end, the frame-wide step schedule over RCCL,
// balanced from calibration frames) and the bands go to rank 0 by sng_gather_rgba8 (RCCL send/recv).
// Rank 0 prints one line per frame and writes PNGs when --out is given.
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/sng.h"

namespace {

struct Options {
    std::string snapshot, virtual_scene, frag, config, scene, out;
    int width = 1280, height = 720;   // main.cu:203-209 defaults
    int sshadows = -1, nshadows = -1;
    int frames = 1, gpus = 1, balance = 4;
    bool display = false, dry_run = false, help = false, version = false, no_gui = false, train = false;
    std::vector<std::pair<std::string, double>> sets;
    std::vector<std::string> files;
};

const char* USAGE =
    "sng-render -- headless SyNeRFgine render path on MI355X (libsng_hip.so)\n"
    "  --snapshot, --load_snapshot PATH  .ingp snapshot (Testbed::load_snapshot)\n"
    "  --virtual, --rt PATH              virtual scene JSON (Engine::set_virtual_world)\n"
    "  --frag PATH                       fragment shader: accepted and ignored (display-only)\n"
    "  --width N, --height N             window resolution (default 1280 x 720)\n"
    "  --sshadows N, --nshadows N        Engine::set_syn_samples / set_nerf_samples\n"
    "  --frames N                        frames to render (default 1)\n"
    "  --out DIR                         write frame-NNNN.png per frame (final RGBA8, or the display stage with --display)\n"
    "  --gpus N                          one process per GPU, row bands + RCCL gather to rank 0 (default 1)\n"
    "  --balance N                       calibration frames that balance the bands (default 4)\n"
    "  --set KEY=VALUE                   engine parameter (sng_set_param), repeatable\n"
    "  --display                         --out through the display stage (main.frag FXAA + blend; --gpus 1)\n"
    "  --dry-run                         print the parsed options as JSON and exit (no GPU)\n"
    "  -h, --help    -v, --version       (--network/--config, --scene, --no-gui, --train, --vr: not on the render path)\n";

bool parse(int argc, char** argv, Options& o, std::string& err) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i], val;
        bool has_val = false;
        const size_t eq = a.find('=');
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            val = a.substr(eq + 1);
            a = a.substr(0, eq);
            has_val = true;
        }
        auto value = [&](std::string& dst) {
            if (has_val) { dst = val; return true; }
            if (i + 1 >= argc) { err = "flag " + a + " needs a value"; return false; }
            dst = argv[++i];
            return true;
        };
        auto number = [&](int& dst) {
            std::string v;
            if (!value(v)) return false;
            char* end = nullptr;
            const long x = std::strtol(v.c_str(), &end, 10);
            if (v.empty() || *end || x < 0 || x > (1L << 30)) { err = "flag " + a + ": bad number '" + v + "'"; return false; }
            dst = (int)x;
            return true;
        };
        if (a == "-h" || a == "--help") o.help = true;
        else if (a == "-v" || a == "--version") o.version = true;
        else if (a == "--snapshot" || a == "--load_snapshot") { if (!value(o.snapshot)) return false; }
        else if (a == "--virtual" || a == "--rt") { if (!value(o.virtual_scene)) return false; }
        else if (a == "--frag") { if (!value(o.frag)) return false; }
        else if (a == "-n" || a == "-c" || a == "--network" || a == "--config") { if (!value(o.config)) return false; }
        else if (a == "-s" || a == "--scene") { if (!value(o.scene)) return false; }
        else if (a == "--width") { if (!number(o.width)) return false; }
        else if (a == "--height") { if (!number(o.height)) return false; }
        else if (a == "--sshadows") { if (!number(o.sshadows)) return false; }
        else if (a == "--nshadows") { if (!number(o.nshadows)) return false; }
        else if (a == "--frames") { if (!number(o.frames)) return false; }
        else if (a == "--gpus") { if (!number(o.gpus)) return false; }
        else if (a == "--balance") { if (!number(o.balance)) return false; }
        else if (a == "--out") { if (!value(o.out)) return false; }
        else if (a == "--set") {
            std::string kv;
            if (!value(kv)) return false;
            const size_t e = kv.find('=');
            char* end = nullptr;
            const double x = e == std::string::npos ? 0.0 : std::strtod(kv.c_str() + e + 1, &end);
            if (e == std::string::npos || e == 0 || !end || *end) { err = "--set needs KEY=VALUE, got '" + kv + "'"; return false; }
            o.sets.emplace_back(kv.substr(0, e), x);
        }
        else if (a == "--display") o.display = true;
        else if (a == "--dry-run") o.dry_run = true;
        else if (a == "--no-gui") o.no_gui = true;
        else if (a == "--train") o.train = true;
        else if (a == "--vr") {}
        else if (a.rfind("-", 0) == 0) { err = "unknown flag " + a; return false; }
        else o.files.push_back(a);
    }
    // positional files (Testbed::load_file, main.cu:172-174): .ingp / .msgpack snapshots, .json scene descriptions
    for (const std::string& f : o.files) {
        auto ends = [&](const char* s) { const size_t n = std::strlen(s); return f.size() >= n && f.compare(f.size() - n, n, s) == 0; };
        if (ends(".ingp") || ends(".msgpack")) o.snapshot = f;
        else if (ends(".json") && o.virtual_scene.empty()) o.virtual_scene = f;
        else { err = "cannot load '" + f + "' on the render path (snapshots and scene JSONs only)"; return false; }
    }
    if (o.width < 1 || o.height < 1) { err = "width and height must be positive"; return false; }
    if (o.gpus < 1) { err = "--gpus must be >= 1"; return false; }
    return true;
}

std::string json_str(const std::string& s) {
    std::string r = "\"";
    for (char ch : s) {
        if (ch == '"' || ch == '\\') r += '\\';
        r += ch;
    }
    return r + "\"";
}

void print_options(const Options& o) {
    std::printf("{\"snapshot\": %s, \"virtual\": %s, \"frag\": %s, \"width\": %d, \"height\": %d, \"sshadows\": %d, \"nshadows\": %d, "
                "\"frames\": %d, \"gpus\": %d, \"balance\": %d, \"out\": %s, \"display\": %s, \"sets\": {",
                json_str(o.snapshot).c_str(), json_str(o.virtual_scene).c_str(), json_str(o.frag).c_str(), o.width, o.height, o.sshadows, o.nshadows,
                o.frames, o.gpus, o.balance, json_str(o.out).c_str(), o.display ? "true" : "false");
    for (size_t k = 0; k < o.sets.size(); ++k) std::printf("%s%s: %.17g", k ? ", " : "", json_str(o.sets[k].first).c_str(), o.sets[k].second);
    std::printf("}}\n");
}

#define CK(call)                                                                                   \
    do {                                                                                           \
        const int rc_ = (call);                                                                    \
        if (rc_ != SNG_OK) {                                                                       \
            std::fprintf(stderr, "sng-render[%d]: %s failed (%d): %s\n", rank, #call, rc_, sng_last_error()); \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

// tiling.balance_bounds: cut the cumulative per-band cost (time / rows, piecewise constant) into equal parts
std::vector<int> balance(int H, const std::vector<int>& b, const std::vector<double>& t, int min_rows = 8, double damping = 0.75) {
    const int W = (int)t.size();
    if (W == 1) return {0, H};
    std::vector<double> dens(W), cum(W + 1, 0.0);
    for (int r = 0; r < W; ++r) dens[r] = std::max(t[r], 1e-6) / std::max(1, b[r + 1] - b[r]);
    for (int r = 0; r < W; ++r) cum[r + 1] = cum[r] + dens[r] * (b[r + 1] - b[r]);
    std::vector<int> n(W + 1, 0);
    for (int k = 1; k < W; ++k) {
        const double target = cum[W] * k / W;
        int r = 0;
        while (r < W - 1 && cum[r + 1] < target) ++r;
        double row = b[r] + (target - cum[r]) / dens[r];
        row = damping * row + (1.0 - damping) * b[k];
        n[k] = (int)std::lround(row);
    }
    n[W] = H;
    const int m = std::min(min_rows, H / W);
    for (int k = 1; k < W; ++k) n[k] = std::max(n[k], n[k - 1] + m);
    for (int k = W - 1; k > 0; --k) n[k] = std::min(n[k], n[k + 1] - m);
    return n;
}

int run_rank(const Options& o, int rank, int world, int id_fd_in, const std::vector<int>& id_fds_out) {
    sng_ctx* ctx = nullptr;
    sng_ctx_desc desc{};
    desc.device_id = rank;
    CK(sng_ctx_create(&desc, &ctx));
    if (!o.snapshot.empty()) CK(sng_load_snapshot(ctx, o.snapshot.c_str()));
    if (!o.virtual_scene.empty()) CK(sng_load_virtual_scene(ctx, o.virtual_scene.c_str()));
    // a camera path in the scene would move the view every frame; the headless frames play it as the reference does
    for (const auto& kv : o.sets) CK(sng_set_param(ctx, kv.first.c_str(), kv.second));
    CK(sng_set_window(ctx, o.width, o.height));
    if (o.sshadows >= 0) {   // main.cu:210-213: both are set when --sshadows is given
        CK(sng_set_param(ctx, "sshadows", (double)o.sshadows));
        CK(sng_set_param(ctx, "nshadows", (double)std::max(0, o.nshadows)));
    }
    sng_resolution_info res{};
    CK(sng_get_resolution(ctx, &res));
    const int MW = res.mesh_res[0], MH = res.mesh_res[1];
    if (world > 1) {
        uint8_t id[SNG_COMM_ID_BYTES];
        if (rank == 0) {
            CK(sng_comm_unique_id(id));
            for (int fd : id_fds_out)
                if (write(fd, id, sizeof(id)) != (ssize_t)sizeof(id)) { std::fprintf(stderr, "sng-render: id pipe write failed\n"); return 1; }
        } else if (read(id_fd_in, id, sizeof(id)) != (ssize_t)sizeof(id)) {
            std::fprintf(stderr, "sng-render[%d]: id pipe read failed\n", rank);
            return 1;
        }
        CK(sng_set_comm(ctx, id, rank, world));
    }
    std::vector<int> bounds(world + 1);
    for (int r = 0; r <= world; ++r) bounds[r] = std::min(MH, r * ((MH + world - 1) / world));
    bounds[world] = MH;
    uint32_t* d_frame = nullptr;   // rank 0: the gathered (or the single-GPU) RGBA8 frame
    uint32_t* d_times = nullptr;
    if (hipSetDevice(rank) != hipSuccess || hipMalloc(&d_frame, (size_t)MW * MH * 4) != hipSuccess ||
        hipMalloc(&d_times, (size_t)world * 4) != hipSuccess) {
        std::fprintf(stderr, "sng-render[%d]: device allocation failed\n", rank);
        return 1;
    }
    sng_frame_params fp{};
    fp.reset_accumulation = 1;
    sng_frame_result fr{};
    // calibration frames: the band split that equalises the per-band device times
    for (int it = 0; world > 1 && it < o.balance; ++it) {
        fp.row_begin = bounds[rank];
        fp.row_end = bounds[rank + 1];
        CK(sng_render_frame(ctx, &fp, &fr));
        std::vector<uint32_t> t(world, 0u);
        t[rank] = (uint32_t)std::lround(fr.ms_frame * 1000.0);
        if (hipMemcpy(d_times, t.data(), world * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
        CK(sng_comm_allreduce_u32(ctx, d_times, world, nullptr));
        CK(sng_synchronize(ctx));
        if (hipMemcpy(t.data(), d_times, world * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        bounds = balance(MH, bounds, std::vector<double>(t.begin(), t.end()));
    }
    if (rank == 0 && !o.out.empty()) mkdir(o.out.c_str(), 0755);
    std::vector<uint32_t> host((size_t)MW * MH);
    std::vector<uint8_t> rgb;
    double total_ms = 0.0;
    for (int f = 0; f < o.frames; ++f) {
        fp.spp = 0;
        fp.row_begin = world > 1 ? bounds[rank] : 0;
        fp.row_end = world > 1 ? bounds[rank + 1] : 0;
        const auto t0 = std::chrono::steady_clock::now();
        CK(sng_render_frame(ctx, &fp, &fr));
        if (world > 1) CK(sng_gather_rgba8(ctx, bounds.data(), rank == 0 ? d_frame : nullptr, nullptr));
        else if (!o.out.empty() && !o.display) CK(sng_final_rgba8(ctx, 0, MH, d_frame, nullptr));
        CK(sng_synchronize(ctx));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        total_ms += ms;
        if (rank != 0) continue;
        std::printf("frame=%d ms=%.3f device_ms=%.3f raytrace_ms=%.3f nerf_ms=%.3f samples=%llu\n", f, ms, fr.ms_frame, fr.ms_raytrace, fr.ms_nerf,
                    (unsigned long long)fr.n_samples);
        if (o.out.empty()) continue;
        char path[4096];
        std::snprintf(path, sizeof(path), "%s/frame-%04d.png", o.out.c_str(), f);
        if (o.display && world == 1) {
            rgb.resize((size_t)o.width * o.height * 3);
            CK(sng_display_frame(ctx, rgb.data(), rgb.size()));
            CK(sng_image_write_png(path, rgb.data(), o.width, o.height, 3));
        } else {
            if (hipMemcpy(host.data(), d_frame, host.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            CK(sng_image_write_png(path, reinterpret_cast<const uint8_t*>(host.data()), MW, MH, 4));
        }
    }
    if (rank == 0)
        std::printf("{\"frames\": %d, \"frames_per_s\": %.3f, \"gpus\": %d, \"width\": %d, \"height\": %d, \"bounds\": [%s]}\n", o.frames,
                    o.frames / (total_ms * 1e-3), world, MW, MH, [&] {
                        std::string s;
                        for (int r = 0; r <= world; ++r) s += (r ? ", " : "") + std::to_string(bounds[r]);
                        return s;
                    }().c_str());
    (void)hipFree(d_frame);
    (void)hipFree(d_times);
    CK(sng_ctx_destroy(ctx));
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    std::string err;
    if (!parse(argc, argv, o, err)) {
        std::fprintf(stderr, "%s\n%s", err.c_str(), USAGE);
        return 2;
    }
    if (o.help) { std::printf("%s", USAGE); return 0; }
    if (o.version) { std::printf("sng-render (libsng_hip ABI %d)\n", sng_abi_version()); return 0; }
    if (o.dry_run) { print_options(o); return 0; }
    if (o.train) { std::fprintf(stderr, "--train: online training runs through sng_train (the Python host mirror); not a render flag\n"); return 2; }
    if (o.gpus == 1) return run_rank(o, 0, 1, -1, {});
    // one process per GPU, forked before anything touches the GPU in this process
    std::vector<int> wr, rd;
    for (int r = 1; r < o.gpus; ++r) {
        int p[2];
        if (pipe(p) != 0) { std::perror("pipe"); return 1; }
        rd.push_back(p[0]);
        wr.push_back(p[1]);
    }
    std::vector<pid_t> kids;
    for (int r = 0; r < o.gpus; ++r) {
        const pid_t pid = fork();
        if (pid < 0) { std::perror("fork"); return 1; }
        if (pid == 0) {
            // keep only this rank's pipe ends: a sibling that dies then closes the last write end of a pipe, so a
            // reader sees EOF instead of blocking forever
            for (int k = 1; k < o.gpus; ++k) {
                if (r != k) close(rd[k - 1]);
                if (r != 0) close(wr[k - 1]);
            }
            const int rc = run_rank(o, r, o.gpus, r > 0 ? rd[r - 1] : -1, r == 0 ? wr : std::vector<int>{});
            std::fflush(stdout);
            _exit(rc);
        }
        kids.push_back(pid);
    }
    for (int k = 1; k < o.gpus; ++k) { close(rd[k - 1]); close(wr[k - 1]); }
    // the first rank that fails ends the run: the others would wait for it in RCCL or in the id pipe
    int worst = 0;
    std::vector<bool> reaped(kids.size(), false);
    for (size_t left = kids.size(); left > 0;) {
        int st = 0;
        const pid_t pid = waitpid(-1, &st, 0);
        if (pid < 0) break;
        for (size_t k = 0; k < kids.size(); ++k)
            if (kids[k] == pid && !reaped[k]) { reaped[k] = true; --left; }
        const int rc = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        if (rc != 0 && worst == 0)
            for (size_t k = 0; k < kids.size(); ++k)
                if (!reaped[k]) kill(kids[k], SIGTERM);
        worst = std::max(worst, rc);
    }
    return worst;
}
