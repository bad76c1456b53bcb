// q2a_group.cpp — one process driving several GPUs through the C ABI (include/q2a_encoder.h, q2a_group_*).
//
// SURVEY.md §8e topology "one process with ncclCommInitAll and a host thread per device": the model is packed ONCE on
// the host into its compact transport form (q2a_pack_model_compact: the file's own ggml rows, 0.38 GB for Q4_K),
// copied to the first device, and sent to every other device by ONE ncclBroadcast over xGMI (RCCL); each device then
// expands it into its own device layout (q2a_open_device_blob). Clips are independent (the reference's encoder has no
// cross-clip state, qwen2-whisper.cpp:2241-2339), so the encode splits a batch into contiguous clip ranges, one host
// thread per device, with no collective on the data path. The reference declares whisper_full_parallel
// (include/qwen2-whisper.h:464-469) but never defines it and initialises a single device
// (whisper_backend_init_gpu, qwen2-whisper.cpp:1217-1279); this is the multi-device path behind it (q2a_whisper.cpp).
#include "q2a_encoder.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" void q2a_internal_set_error(const char * msg);

extern "C" int q2a_internal_engine_blob(const q2a_engine * e, const void ** blob, int64_t * bytes, int * device);

struct q2a_group {
    std::vector<int> dev;
    std::vector<q2a_engine *> eng;
    // q2a_group_open_with: the received device-layout replicas the other devices' engines run on (they do not own
    // them), released after those engines
    std::vector<std::pair<int, void *>> held;
    int64_t blob_bytes = 0;
    double t_pack = 0, t_bcast = 0, t_open = 0;   // seconds: host pack, H2D + RCCL broadcast, expand / engine open
};

namespace {

void gerr(const char * fmt, ...) __attribute__((format(printf, 1, 2)));
void gerr(const char * fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    q2a_internal_set_error(buf);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// device buffers and streams of the broadcast, released on every path out of q2a_group_open
struct bcast_bufs {
    std::vector<int> dev;
    std::vector<void *> buf;
    std::vector<hipStream_t> st;
    std::vector<ncclComm_t> comm;
    ~bcast_bufs() {
        for (size_t i = 0; i < dev.size(); ++i) {
            (void) hipSetDevice(dev[i]);
            if (i < st.size() && st[i]) (void) hipStreamSynchronize(st[i]);
            if (i < buf.size() && buf[i]) (void) hipFree(buf[i]);
            if (i < st.size() && st[i]) (void) hipStreamDestroy(st[i]);
        }
        for (ncclComm_t c : comm)
            if (c) (void) ncclCommDestroy(c);
    }
};

int q2a_device_count_impl() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void) hipGetLastError(); return 0; }
    return n;
}

int q2a_group_split_impl(int n_clips, int n_devices, int i, int * first, int * count) {
    if (n_clips < 0 || n_devices <= 0 || i < 0 || i >= n_devices || !first || !count) {
        gerr("invalid arguments");
        return Q2A_ERR_ARG;
    }
    // contiguous near-equal ranges, the first n_clips % n_devices one clip longer (q2a/dist.py split_batch)
    const int base = n_clips / n_devices, extra = n_clips % n_devices;
    *first = i * base + (i < extra ? i : extra);
    *count = base + (i < extra ? 1 : 0);
    return Q2A_OK;
}

// the device list of a group: devices[0..n) checked (in range, no repeats), or every visible device when n == 0 (with
// `first` moved to the front when >= 0)
bool group_devices(const int * devices, int n_devices, int first, std::vector<int> & dev) {
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible <= 0) {
        (void) hipGetLastError();
        gerr("no HIP device available");
        return false;
    }
    dev.clear();
    if (n_devices == 0) {
        if (first >= 0) dev.push_back(first);
        for (int d = 0; d < visible; ++d)
            if (d != first) dev.push_back(d);
    } else {
        dev.assign(devices, devices + n_devices);
    }
    for (size_t i = 0; i < dev.size(); ++i) {
        if (dev[i] < 0 || dev[i] >= visible) { gerr("device %d not available (%d devices)", dev[i], visible); return false; }
        for (size_t j = 0; j < i; ++j)
            if (dev[j] == dev[i]) { gerr("device %d listed twice", dev[i]); return false; }
    }
    return true;
}

// ONE grouped ncclBroadcast of nb bytes from src (on dev[root]) into b.buf[i] of every other device (communicators from
// ncclCommInitAll over dev, rank i = dev[i]); b.buf[root] must be src. Q2A_OK when every device's copy has landed.
int broadcast(bcast_bufs & b, const std::vector<int> & dev, int root, int64_t nb) {
    const int n = (int) dev.size();
    b.comm.assign(n, nullptr);
    ncclResult_t r = ncclCommInitAll(b.comm.data(), n, dev.data());
    if (r != ncclSuccess) { gerr("ncclCommInitAll over %d devices: %s", n, ncclGetErrorString(r)); return Q2A_ERR_HIP; }
    r = ncclGroupStart();
    for (int i = 0; i < n && r == ncclSuccess; ++i) {
        (void) hipSetDevice(dev[i]);
        r = ncclBroadcast(b.buf[root], b.buf[i], (size_t) nb, ncclUint8, root, b.comm[i], b.st[i]);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) {
        gerr("ncclBroadcast of the weight blob: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
        return Q2A_ERR_HIP;
    }
    for (int i = 0; i < n; ++i)
        if (hipSetDevice(dev[i]) != hipSuccess || hipStreamSynchronize(b.st[i]) != hipSuccess) {
            gerr("device %d: broadcast did not complete", dev[i]);
            return Q2A_ERR_HIP;
        }
    return Q2A_OK;
}

// one stream per device and an nb-byte receive buffer on every device but `skip` (-1: on every device)
int alloc_bufs(bcast_bufs & b, const std::vector<int> & dev, int64_t nb, int skip) {
    const int n = (int) dev.size();
    b.dev = dev;
    b.buf.assign(n, nullptr);
    b.st.assign(n, nullptr);
    for (int i = 0; i < n; ++i) {
        if (hipSetDevice(dev[i]) != hipSuccess || hipStreamCreateWithFlags(&b.st[i], hipStreamNonBlocking) != hipSuccess) {
            gerr("device %d: stream creation failed", dev[i]);
            return Q2A_ERR_HIP;
        }
        if (i != skip && hipMalloc(&b.buf[i], (size_t) nb) != hipSuccess) {
            (void) hipGetLastError();
            gerr("device %d: %.2f GB for the weight blob", dev[i], nb / 1e9);
            return Q2A_ERR_OOM;
        }
    }
    return Q2A_OK;
}

}  // namespace

extern "C" {

int q2a_device_count(void) { return q2a_device_count_impl(); }

int q2a_group_split(int n_clips, int n_devices, int i, int * first, int * count) {
    return q2a_group_split_impl(n_clips, n_devices, i, first, count);
}

q2a_group * q2a_group_open(const char * model_path, const int * devices, int n_devices, int act) {
    if (!model_path || n_devices < 0 || (n_devices > 0 && !devices)) { gerr("invalid arguments"); return nullptr; }
    std::vector<int> dev;
    if (!group_devices(devices, n_devices, -1, dev)) return nullptr;
    const int n = (int) dev.size();
    q2a_group * g = new q2a_group();
    g->dev = dev;
    double t0 = now_s();
    void * host = nullptr;
    const int64_t nb = q2a_pack_model_compact(model_path, act, &host);
    if (nb < 0) { delete g; return nullptr; }   // (the packer set the message)
    g->blob_bytes = nb;
    g->t_pack = now_s() - t0;
    t0 = now_s();
    int rc = Q2A_OK;
    {
        bcast_bufs b;
        rc = alloc_bufs(b, dev, nb, -1);
        if (rc == Q2A_OK && (hipSetDevice(dev[0]) != hipSuccess ||
                             hipMemcpy(b.buf[0], host, (size_t) nb, hipMemcpyHostToDevice) != hipSuccess)) {
            gerr("weight upload to device %d failed", dev[0]);
            rc = Q2A_ERR_HIP;
        }
        q2a_free_host_blob(host);
        host = nullptr;
        // one communicator clique over the listed devices, rank i = dev[i]; rank 0 holds the blob
        if (rc == Q2A_OK) rc = broadcast(b, dev, 0, nb);
        g->t_bcast = now_s() - t0;
        t0 = now_s();
        // every device expands its copy into an engine-owned device layout (k_expand_rows), then the transport copy
        // is released with the bcast_bufs
        for (int i = 0; i < n && rc == Q2A_OK; ++i) {
            q2a_engine * e = q2a_open_device_blob(b.buf[i], nb, dev[i]);
            if (!e) { rc = Q2A_ERR_HIP; break; }
            g->eng.push_back(e);
        }
        g->t_open = now_s() - t0;
    }
    if (rc != Q2A_OK) {
        const std::string msg = q2a_last_error();
        q2a_group_close(g);
        q2a_internal_set_error(msg.c_str());
        return nullptr;
    }
    return g;
}

q2a_group * q2a_group_open_with(q2a_engine * base, const int * devices, int n_devices) {
    const void * src = nullptr;
    int64_t nb = 0;
    int bdev = -1;
    if (!base || n_devices < 0 || (n_devices > 0 && !devices)) { gerr("invalid arguments"); return nullptr; }
    if (q2a_internal_engine_blob(base, &src, &nb, &bdev) != Q2A_OK) return nullptr;
    std::vector<int> dev;
    if (!group_devices(devices, n_devices, bdev, dev)) return nullptr;
    int root = -1;
    for (int i = 0; i < (int) dev.size(); ++i)
        if (dev[i] == bdev) root = i;
    if (root < 0) { gerr("the base engine's device %d is not in the device list", bdev); return nullptr; }
    const int n = (int) dev.size();
    q2a_group * g = new q2a_group();
    g->dev = dev;
    g->blob_bytes = nb;
    double t0 = now_s();
    int rc = Q2A_OK;
    {
        bcast_bufs b;
        rc = alloc_bufs(b, dev, nb, root);
        if (rc == Q2A_OK) {
            b.buf[root] = const_cast<void *>(src);   // the base engine's own replica is the broadcast's source (read only)
            if (n > 1) rc = broadcast(b, dev, root, nb);
        }
        g->t_bcast = now_s() - t0;
        t0 = now_s();
        // the base device's engine shares base's weights (its own workspace and stream); every other device's engine
        // runs on the replica it received, which the group keeps until close
        for (int i = 0; i < n && rc == Q2A_OK; ++i) {
            q2a_engine * e = i == root ? q2a_open_shared(base) : q2a_open_device_blob(b.buf[i], nb, dev[i]);
            if (!e) { rc = Q2A_ERR_HIP; break; }
            g->eng.push_back(e);
            if (i != root) { g->held.emplace_back(dev[i], b.buf[i]); b.buf[i] = nullptr; }
        }
        b.buf[root] = nullptr;   // (never freed here: it belongs to base)
        g->t_open = now_s() - t0;
    }
    if (rc != Q2A_OK) {
        const std::string msg = q2a_last_error();
        q2a_group_close(g);
        q2a_internal_set_error(msg.c_str());
        return nullptr;
    }
    return g;
}

int q2a_group_size(const q2a_group * g) { return g ? (int) g->eng.size() : 0; }

q2a_engine * q2a_group_engine(q2a_group * g, int i) {
    if (!g || i < 0 || i >= (int) g->eng.size()) { gerr("invalid arguments"); return nullptr; }
    return g->eng[i];
}

int q2a_group_setup_times(const q2a_group * g, double * pack_s, double * broadcast_s, double * open_s, int64_t * blob_bytes) {
    if (!g) { gerr("invalid arguments"); return Q2A_ERR_ARG; }
    if (pack_s) *pack_s = g->t_pack;
    if (broadcast_s) *broadcast_s = g->t_bcast;
    if (open_s) *open_s = g->t_open;
    if (blob_bytes) *blob_bytes = g->blob_bytes;
    return Q2A_OK;
}

int q2a_group_encode_host(q2a_group * g, const float * const * pcm, const int32_t * n_samples, const int32_t * offsets_ms,
                          int n_clips, int offset_ms, float * out_host, int32_t * status) {
    if (!g || g->eng.empty() || !pcm || !n_samples || !out_host || n_clips <= 0) { gerr("invalid arguments"); return Q2A_ERR_ARG; }
    q2a_info info;
    if (q2a_get_info(g->eng[0], &info) != Q2A_OK) return Q2A_ERR_ARG;
    const size_t per_out = (size_t) info.n_out * info.n_audio_state;
    const int n = (int) g->eng.size();
    std::vector<int> rcs(n, Q2A_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) {
        int f = 0, c = 0;
        q2a_group_split(n_clips, n, i, &f, &c);
        if (c == 0) continue;
        // one host thread per device: each runs the chunked, copy-overlapped host path of its own engine on its range
        th.emplace_back([&, i, f, c]() {
            rcs[i] = q2a_encode_host_ex(g->eng[i], pcm + f, n_samples + f, offsets_ms ? offsets_ms + f : nullptr, c, offset_ms,
                                        out_host + (size_t) f * per_out, status ? status + f : nullptr);
            if (rcs[i] != Q2A_OK) msg[i] = q2a_last_error();
        });
    }
    for (auto & t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rcs[i] != Q2A_OK) {
            gerr("device %d: %s", g->dev[i], msg[i].c_str());
            return rcs[i];
        }
    return Q2A_OK;
}

void q2a_group_close(q2a_group * g) {
    if (!g) return;
    for (q2a_engine * e : g->eng) q2a_close(e);
    for (auto & h : g->held) {
        (void) hipSetDevice(h.first);
        (void) hipFree(h.second);
    }
    delete g;
}

}  // extern "C"
