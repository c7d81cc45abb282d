// Frame-wide step schedule across GPUs: the one exchange of the band-sharded
// path.  trace_alt sizes every iteration from the frame-wide alive count
// (testbed_nerf.cu:2180-2190); with one band per GPU that count is the sum over ranks, formed
// here by an in-place RCCL all-reduce of one uint32 on the NeRF stream (no host round trip).
//
// RCCL is opened lazily with dlopen when a communicator is attached, so the library carries no
// link-time RCCL dependency and, inside a PyTorch process, binds to the RCCL that torch already
// loaded (same soname, librccl.so.1) instead of a second copy.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "sng_internal.h"

namespace sng {

namespace {
struct RcclApi {
    void* lib = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        a.lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!a.lib) a.lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!a.lib) return a;
        a.get_unique_id = reinterpret_cast<decltype(&ncclGetUniqueId)>(dlsym(a.lib, "ncclGetUniqueId"));
        a.comm_init_rank = reinterpret_cast<decltype(&ncclCommInitRank)>(dlsym(a.lib, "ncclCommInitRank"));
        a.comm_destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(a.lib, "ncclCommDestroy"));
        a.all_reduce = reinterpret_cast<decltype(&ncclAllReduce)>(dlsym(a.lib, "ncclAllReduce"));
        a.send = reinterpret_cast<decltype(&ncclSend)>(dlsym(a.lib, "ncclSend"));
        a.recv = reinterpret_cast<decltype(&ncclRecv)>(dlsym(a.lib, "ncclRecv"));
        a.group_start = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(a.lib, "ncclGroupStart"));
        a.group_end = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(a.lib, "ncclGroupEnd"));
        a.error_string = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(a.lib, "ncclGetErrorString"));
        return a;
    }();
    if (!api.lib || !api.get_unique_id || !api.comm_init_rank || !api.comm_destroy || !api.all_reduce || !api.send || !api.recv ||
        !api.group_start || !api.group_end || !api.error_string)
        throw SngError(SNG_ERR_STATE, std::string("RCCL (librccl.so.1) not loadable: ") + (dlerror() ? dlerror() : "missing symbols"));
    return api;
}

void check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw SngError(SNG_ERR_HIP, std::string(what) + ": " + rccl().error_string(r));
}
}  // namespace

void comm_unique_id(uint8_t out[SNG_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == SNG_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    std::memcpy(out, &id, sizeof(id));
}

void comm_init(SchedComm& c, const uint8_t* id, int rank, int world) {
    comm_destroy(c);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    check(rccl().comm_init_rank(&comm, world, uid, rank), "ncclCommInitRank");
    c.comm = comm;
    c.rank = rank;
    c.world = world;
}

void comm_destroy(SchedComm& c) {
    if (c.comm) {
        ncclComm_t comm = static_cast<ncclComm_t>(c.comm);
        c.comm = nullptr;
        (void)rccl().comm_destroy(comm);
    }
    c.rank = 0;
    c.world = 0;
}

void comm_allreduce_u32(SchedComm& c, const uint32_t* src, uint32_t* dst, size_t n, hipStream_t s) {
    check(rccl().all_reduce(src, dst, n, ncclUint32, ncclSum, static_cast<ncclComm_t>(c.comm), s), "ncclAllReduce");
}

// The final composition: every rank's band of RGBA8 rows goes to the root rank only -- one
// grouped ncclSend per peer, ncclRecv of each band straight into its rows of the root's frame (the
// reference's only per-view copy-back is testbed.cu:5126-5127).  offsets / sizes: bytes per rank.
void comm_gather_to_root(SchedComm& c, const void* d_band, void* d_frame, const size_t* offsets, const size_t* sizes, hipStream_t s) {
    const RcclApi& r = rccl();
    ncclComm_t comm = static_cast<ncclComm_t>(c.comm);
    if (c.rank == 0) {
        if (sizes[0] && hipMemcpyAsync(static_cast<uint8_t*>(d_frame) + offsets[0], d_band, sizes[0], hipMemcpyDeviceToDevice, s) != hipSuccess)
            throw SngError(SNG_ERR_HIP, "gather: local band copy failed");
        check(r.group_start(), "ncclGroupStart");
        for (int k = 1; k < c.world; ++k)
            if (sizes[k]) check(r.recv(static_cast<uint8_t*>(d_frame) + offsets[k], sizes[k], ncclUint8, k, comm, s), "ncclRecv");
        check(r.group_end(), "ncclGroupEnd");
    } else if (sizes[c.rank]) {
        check(r.send(d_band, sizes[c.rank], ncclUint8, 0, comm, s), "ncclSend");
    }
}

}  // namespace sng
