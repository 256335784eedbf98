// rtw_multi.cpp -- rendering::render on several GPUs of one node from one caller (C ABI).
//
// The reference's render (src/lib/rendering.rs:121-220) is one call that uses every core; SURVEY §8(b)
// asks its replacement to take the node's devices the same way ("one call may use several devices
// internally").  A frame here is cut into the interleaved 8x8 tiles of DESIGN §7: entry i of the
// device list renders the tiles t with t % n == i (rtw_render_device, RTW_LAYOUT_TILES) on its own
// host thread and stream, its tile buffer reaches devices[0] by a peer copy over xGMI, and
// rtw_untile_device places every partition's tiles there.  Per-(pixel, sample) RNG streams make the
// image independent of the partition, so it equals rtw_render's bit for bit.
// A device may appear several times (several partitions on one GPU; the tests use {0, 0, 0}).
// Built only on the public ABI of include/rtw.h: no kernel internals here.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "rtw_common.h"

struct rtw_multi {
    std::vector<int> devices;          // partition i renders on devices[i]
    std::vector<rtw_gpu_world*> worlds;  // one resident world per partition (its own queue and buffers)
    std::vector<hipStream_t> streams;  // one per partition, on its device
    std::vector<float*> tiles;         // partition i's tile buffer, on devices[i]
    std::vector<size_t> tile_floats;   // ... and its size
    float* gather = nullptr;           // n x stride floats on devices[0]
    size_t gather_floats = 0;
    float* image = nullptr;            // W x H x 3 on devices[0] (rtw_render_devices' own frame)
    size_t image_floats = 0;
    // RTW_MULTI_FORCE_PEER=1 at create: partitions on devices[0] too copy with hipMemcpyPeerAsync (a
    // same-device peer copy), so the one-GPU box runs the copy distinct devices take
    bool force_peer = false;
    std::atomic<uint64_t> peer_copies{0};  // hipMemcpyPeerAsync calls so far (rtw_multi_peer_copies)
};

namespace {

#define MT_TRY(expr)                                                                              \
    do {                                                                                          \
        const hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return rtw::fail(RTW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int grow_on(int device, float** buf, size_t* have, size_t floats) {
    if (*have >= floats) return RTW_OK;
    MT_TRY(hipSetDevice(device));
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    const hipError_t e = hipMalloc((void**)buf, std::max<size_t>(floats, 1) * sizeof(float));
    if (e != hipSuccess) return rtw::fail(RTW_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    *have = floats;
    return RTW_OK;
}

// the render parameters of partition i of n (validated copies of the caller's)
rtw_render_params part_params(const rtw_render_params* p, int i, int n) {
    rtw_render_params q = *p;
    q.layout = RTW_LAYOUT_TILES;
    q.part_index = i;
    q.part_count = n;
    return q;
}

}  // namespace

extern "C" RTW_API int rtw_multi_release(rtw_multi* m) {
    if (!m) return RTW_OK;
    for (size_t i = 0; i < m->devices.size(); ++i) {
        (void)hipSetDevice(m->devices[i]);
        if (i < m->streams.size() && m->streams[i]) {
            (void)hipStreamSynchronize(m->streams[i]);
            (void)hipStreamDestroy(m->streams[i]);
        }
        if (i < m->tiles.size() && m->tiles[i]) (void)hipFree(m->tiles[i]);
        if (i < m->worlds.size()) rtw_world_release(m->worlds[i]);
    }
    if (!m->devices.empty()) {
        (void)hipSetDevice(m->devices[0]);
        if (m->gather) (void)hipFree(m->gather);
        if (m->image) (void)hipFree(m->image);
    }
    delete m;
    return RTW_OK;
}

extern "C" RTW_API int rtw_multi_create(const rtw_world* world, const int* devices, int n_devices, rtw_multi** out) {
    if (!out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!world || !devices) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    if (n_devices < 1) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "n_devices must be >= 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device: the MI355X path requires a GPU (there is no CPU fallback)");
    for (int i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= ndev) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "device index out of range");
    auto* m = new rtw_multi;
    if (const char* e = std::getenv("RTW_MULTI_FORCE_PEER")) m->force_peer = e[0] == '1';
    m->devices.assign(devices, devices + n_devices);
    m->worlds.assign((size_t)n_devices, nullptr);
    m->streams.assign((size_t)n_devices, nullptr);
    m->tiles.assign((size_t)n_devices, nullptr);
    m->tile_floats.assign((size_t)n_devices, 0);
    const int d0 = devices[0];
    for (int i = 0; i < n_devices; ++i) {
        const int d = devices[i];
        int rc = rtw_world_upload(world, d, &m->worlds[(size_t)i]);
        if (rc == RTW_OK && hipSetDevice(d) != hipSuccess) rc = rtw::fail(RTW_ERR_HIP, "hipSetDevice");
        if (rc == RTW_OK && hipStreamCreateWithFlags(&m->streams[(size_t)i], hipStreamNonBlocking) != hipSuccess)
            rc = rtw::fail(RTW_ERR_HIP, "hipStreamCreate");
        // the tile copies go from device d straight into devices[0]'s memory over xGMI when the
        // pair allows peer access (otherwise hipMemcpyPeerAsync stages them)
        if (rc == RTW_OK && d != d0) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, d, d0) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(d0, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                    rc = rtw::fail(RTW_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                }
                (void)hipGetLastError();  // clear an "already enabled" status
            }
        }
        if (rc != RTW_OK) {
            rtw_multi_release(m);
            return rc;
        }
    }
    *out = m;
    return RTW_OK;
}

// One frame on every partition; the image (W*H*3 f32, row-major from the top-left pixel) lands in
// d_image on devices[0].  Synchronous: returns when the image is complete.
extern "C" RTW_API int rtw_multi_render(rtw_multi* m, const rtw_render_params* params, float* d_image) {
    if (!m || !params || !d_image) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    if (params->part_count > 1 || params->part_index != 0)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_multi_render partitions the frame itself: part_count must be 0 or 1");
    const int n = (int)m->devices.size();
    // every partition's buffer padded to partition 0's size (the largest): the untile kernel's stride
    int64_t stride = 0;
    {
        const rtw_render_params q = part_params(params, 0, n);
        const int rc = rtw_partition_floats(&q, &stride);
        if (rc != RTW_OK) return rc;
    }
    for (int i = 0; i < n; ++i) {
        const int rc = grow_on(m->devices[(size_t)i], &m->tiles[(size_t)i], &m->tile_floats[(size_t)i], (size_t)stride);
        if (rc != RTW_OK) return rc;
    }
    {
        const int rc = grow_on(m->devices[0], &m->gather, &m->gather_floats, (size_t)stride * (size_t)n);
        if (rc != RTW_OK) return rc;
    }
    // one host thread per partition: render its tiles, copy them into slot i of the gather buffer
    std::vector<int> rcs((size_t)n, RTW_OK);
    std::vector<std::string> errs((size_t)n);
    auto work = [&](int i) {
        const int d = m->devices[(size_t)i], d0 = m->devices[0];
        hipStream_t s = m->streams[(size_t)i];
        auto failed = [&](int code, const std::string& msg) {
            rcs[(size_t)i] = code;
            errs[(size_t)i] = msg;
        };
        if (hipSetDevice(d) != hipSuccess) return failed(RTW_ERR_HIP, "hipSetDevice");
        const rtw_render_params q = part_params(params, i, n);
        int64_t floats = 0;
        int rc = rtw_partition_floats(&q, &floats);
        if (rc == RTW_OK) rc = rtw_render_device(m->worlds[(size_t)i], &q, m->tiles[(size_t)i], (void*)s);
        if (rc != RTW_OK) return failed(rc, rtw_last_error());
        float* dst = m->gather + (size_t)i * (size_t)stride;
        const size_t bytes = (size_t)floats * sizeof(float);
        const bool peer = d != d0 || m->force_peer;
        hipError_t e = bytes == 0 ? hipSuccess
                       : !peer    ? hipMemcpyAsync(dst, m->tiles[(size_t)i], bytes, hipMemcpyDeviceToDevice, s)
                                  : hipMemcpyPeerAsync(dst, d0, m->tiles[(size_t)i], d, bytes, s);
        if (bytes != 0 && peer && e == hipSuccess) m->peer_copies.fetch_add(1, std::memory_order_relaxed);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return failed(RTW_ERR_HIP, std::string("partition copy: ") + hipGetErrorString(e));
    };
    if (n == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        th.reserve((size_t)n);
        for (int i = 0; i < n; ++i) th.emplace_back(work, i);
        for (std::thread& t : th) t.join();
    }
    for (int i = 0; i < n; ++i)
        if (rcs[(size_t)i] != RTW_OK) return rtw::fail(rcs[(size_t)i], "partition " + std::to_string(i) + ": " + errs[(size_t)i]);
    MT_TRY(hipSetDevice(m->devices[0]));
    rtw_render_params q = *params;
    q.part_index = 0;
    q.part_count = n;
    const int rc = rtw_untile_device(&q, m->gather, stride, d_image, (void*)m->streams[0]);
    if (rc != RTW_OK) return rc;
    MT_TRY(hipStreamSynchronize(m->streams[0]));
    return RTW_OK;
}

extern "C" RTW_API int rtw_multi_peer_copies(const rtw_multi* m, uint64_t* copies) {
    if (!m || !copies) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    *copies = m->peer_copies.load(std::memory_order_relaxed);
    return RTW_OK;
}

extern "C" RTW_API int rtw_render_devices(const rtw_world* world, const rtw_render_params* params, const int* devices,
                                          int n_devices, float* out_rgb) {
    if (!params || !out_rgb) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    if (params->width < 2 || params->height < 2)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "image width and height must be >= 2");
    rtw_multi* m = nullptr;
    int rc = rtw_multi_create(world, devices, n_devices, &m);
    if (rc != RTW_OK) return rc;
    const size_t floats = (size_t)params->width * (size_t)params->height * 3;
    rc = grow_on(m->devices[0], &m->image, &m->image_floats, floats);
    if (rc == RTW_OK) {
        rtw_render_params q = *params;
        q.part_index = 0;
        q.part_count = 1;
        rc = rtw_multi_render(m, &q, m->image);
    }
    if (rc == RTW_OK) {
        const hipError_t e = hipMemcpy(out_rgb, m->image, floats * sizeof(float), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = rtw::fail(RTW_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    rtw_multi_release(m);
    return rc;
}
