// async.cpp — vr::AsyncMultiMapper (modules/octvr/src/async.cpp:32-350) on one device.
//
// Same five-stage pipeline as the reference — host planes -> pinned staging -> device upload ->
// stitch of every mapper -> device download -> pinned -> host output planes — over a ring of
// kSlots buffer sets, so consecutive frames overlap (frame k+2 is copied in while k+1 uploads and
// k is stitched).  Differences from the reference, all deliberate:
//   * one HIP stream per stage (upload, compute, download), never the legacy default stream;
//   * gain chaining (gain_modes[i] = j < i) copies mapper j's device gains on the compute stream
//     instead of round-tripping them through the host (async.cpp:78-86);
//   * worker threads are joinable and exit when the object is destroyed (the reference's five
//     threads loop forever and its destructor clears joinable std::threads, async.cpp:87-90,337-349);
//   * a failing frame carries its status to pop() instead of asserting;
//   * the two host-copy stages split their rows over a few helper threads (RowPool): one thread's
//     memcpy from pageable memory (~15 GB/s) otherwise bounds the whole pipeline (scripts/async_trace.py);
//   * only the input bytes some kernel of some mapper reads are copied and uploaded (the union of the
//     mappers' source footprints, host_common.hpp SourceFootprint), packed, and put in place on the
//     device by one kernel: with the copy chain each output pixel comes from one camera, so a C2 frame
//     needs ~18 MB of its 75 MB of YUV (the composite's staged groups plus the gain samples' row pairs,
//     DESIGN.md §6);
//   * output planes the caller registers once (octvr_async_register_output: a ring it reuses, as the
//     reference's own output Mats are reused, async.cpp:113-138) are page-locked and written by the D2H
//     copies directly, region by region (2-D copies at the caller's pitch): no pinned staging and no
//     copy-out for them; other planes take the staging path;
//   * the preview (async.cpp:73-110, 141-171) is published to a caller-read buffer and an optional sink
//     (octvr_async_pop_preview / octvr_async_set_preview_sink) instead of Qt shared memory, which stays
//     the caller's.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host_common.hpp"

using namespace octvr;

namespace {

constexpr int kSlots = 3;  // BUF_SIZE (async.cpp:261)

template <class T>
class Channel {  // blocking FIFO; close() wakes every waiter, pop() then drains what is left
public:
    void push(T v) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(v));
        }
        cv_.notify_one();
    }
    bool pop(T& out) {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return false;
        out = std::move(q_.front());
        q_.pop_front();
        return true;
    }
    void close() {
        {
            std::lock_guard<std::mutex> g(mu_);
            closed_ = true;
        }
        cv_.notify_all();
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<T> q_;
    bool closed_ = false;
};

struct Rect {
    int x, y, w, h;
};

// _rect_mul_size (async.cpp:20-30)
Rect rect_mul_size(const double* r, int W, int H) {
    Rect o{(int)std::round(r[0] * W), (int)std::round(r[1] * H), (int)std::round(r[2] * W), (int)std::round(r[3] * H)};
    if (o.x + o.w >= W) o.w = W - o.x;
    if (o.y + o.h >= H) o.h = H - o.y;
    return o;
}

struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    void alloc(size_t bytes) {
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p), bytes, hipHostMallocDefault));
        n = bytes;
    }
};

struct Slot {  // one frame's buffers: the packed footprint runs, the device frames ("Y over [U|V]", pitch = width)
    std::unique_ptr<PinnedBuf> packed_host;
    DevBuf<uint8_t> packed_dev;
    DevBuf<uint8_t> preview_dev;  // preview_w x preview_h RGB, black outside the regions (async.cpp:314-316)
    std::unique_ptr<PinnedBuf> preview_host;
    std::vector<std::unique_ptr<PinnedBuf>> out_host;
    std::vector<DevBuf<uint8_t>> in_dev, out_dev;
    FootFrames frames{};
};

// Runs of the union of the mappers' footprints: per camera and row pair, consecutive set groups, gaps of
// up to kRunGap groups bridged (a few more bytes for fewer, longer copies)
constexpr int kRunGap = 2;
std::vector<FootRun> footprint_runs(const SourceFootprint& f, size_t& bytes) {
    std::vector<FootRun> runs;
    bytes = 0;
    for (int i = 0; i < (int)f.w.size(); i++)
        for (int r = 0; r < f.row_pairs(i); r++) {
            int g = 0;
            const int G = f.groups(i);
            while (g < G) {
                if (!f.test(i, r, g)) {
                    g++;
                    continue;
                }
                int e = g + 1, last = g;  // last set group of the run
                while (e < G && e - last <= kRunGap + 1) {
                    if (f.test(i, r, e)) last = e;
                    e++;
                }
                const int ng = last - g + 1;
                const int yb = std::min(8 * (g + ng), f.w[i]) - 8 * g;
                const int cb = std::max(0, std::min(4 * (g + ng), f.w[i] / 2) - 4 * g);
                runs.push_back(FootRun{(uint32_t)i | (uint32_t)r << 8, (uint32_t)g, (uint32_t)ng, (uint32_t)bytes});
                bytes += (size_t)(2 * yb + 2 * cb);
                g = last + 1;
            }
        }
    return runs;
}

struct Job {
    std::vector<const uint8_t*> in_planes;
    std::vector<size_t> in_pitches;
    uint8_t* out_planes[3] = {nullptr, nullptr, nullptr};
    size_t out_pitches[3] = {0, 0, 0};
    bool direct = false;  // the output planes are registered: the D2H writes them, no copy-out
    int slot = -1;
    int status = OCTVR_OK;
    std::string error;
};

// Helper threads of one host-copy stage: run(n, f) calls f(lo, hi) over n rows split into contiguous
// ranges, the calling thread taking the last one, and returns when all are done.  One run at a time
// (each stage owns its pool); f must not throw (memcpy only).
class RowPool {
public:
    explicit RowPool(int helpers) {
        for (int i = 0; i < helpers; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~RowPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    template <class F>
    void run(size_t n, F f) {
        const size_t T = th_.size() + 1;
        std::function<void(size_t, size_t)> fn = f;
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            n_ = n;
            left_ = th_.size();
            gen_++;
        }
        cv_.notify_all();
        fn(n * (T - 1) / T, n);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return left_ == 0; });
        job_ = nullptr;
    }

private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t, size_t)>* f;
            size_t n, T;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                f = job_;
                n = n_;
                T = th_.size() + 1;
            }
            (*f)(n * (size_t)i / T, n * (size_t)(i + 1) / T);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--left_ == 0) done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t, size_t)>* job_ = nullptr;
    size_t n_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};
constexpr int kCopyHelpers = 5;  // per host-copy stage (the GPU box grants ~16 host threads per GPU)

template <class F>
void stage(Job& j, F&& f) {  // run a stage unless the frame already failed; record the first failure
    if (j.status != OCTVR_OK) return;
    try {
        f();
    } catch (const OctvrError& e) {
        j.status = e.code;
        j.error = e.what();
    } catch (const std::exception& e) {
        j.status = OCTVR_E_HIP;
        j.error = e.what();
    }
}

}  // namespace

struct octvr_async {
    int device = 0;
    int n_in = 0;
    int out_w = 0, out_h = 0;
    std::vector<int> in_w, in_h;
    std::vector<octvr_mapper*> mappers;
    std::vector<int> gain_modes;
    std::vector<Rect> regions, regions_uv;  // per mapper: its rectangle in the Y and in the U / V planes
    int flags = 0;
    // preview (async.cpp:73-76): preview_w x preview_h RGB; per mapper its rectangle (w or h <= 0: none)
    int preview_w = 0, preview_h = 0;
    std::vector<Rect> preview_rects;
    std::mutex pub_mu;  // the published preview, its header and the sink
    std::vector<uint8_t> pub;
    octvr_preview_header pub_hdr{0, 0, 0, 0.0};
    octvr_preview_sink sink = nullptr;
    void* sink_user = nullptr;
    // fps over blocks of 10 frames, as the reference's copy-out thread keeps it (async.cpp:141-147): the
    // frame interval is measured from the previous frame's copy-out (the first from creation, fps_timer)
    std::chrono::steady_clock::time_point fps_t = std::chrono::steady_clock::now();
    int64_t frame_count = 0;
    double frame_total_ms = 0, frame_fps = 0;
    std::vector<FootRun> runs;  // what the mappers read of the inputs (footprint_runs)
    size_t packed_bytes = 0;
    DevBuf<FootRun> runs_dev;
    Slot slots[kSlots];
    // output plane sets the caller registered (octvr_async_register_output): page-locked, downloaded into
    struct RegOut {
        uint8_t* p[3];
        size_t pitch[3];
    };
    std::vector<RegOut> reg_out;  // caller thread only (register / push / destroy)
    hipStream_t up = nullptr, comp = nullptr, down = nullptr;
    Channel<std::shared_ptr<Job>> q_in, q_up, q_map, q_down, q_out, q_done;
    Channel<int> free_slots;
    std::vector<std::thread> threads;
    RowPool copy_in_pool{kCopyHelpers}, copy_out_pool{kCopyHelpers};
    int pending = 0;  // pushed, not popped (caller thread only)

    ~octvr_async() {
        q_in.close();
        for (auto& t : threads)
            if (t.joinable()) t.join();
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (const RegOut& r : reg_out)
            for (uint8_t* p : r.p) (void)hipHostUnregister(p);
        for (hipStream_t s : {up, comp, down})
            if (s) (void)hipStreamDestroy(s);
        for (auto& sl : slots) {
            sl.in_dev.clear();
            sl.out_dev.clear();
            sl.packed_dev.reset();
            sl.packed_host.reset();
            sl.preview_dev.reset();
            sl.preview_host.reset();
            sl.out_host.clear();
        }
        for (auto* m : mappers) octvr_mapper_destroy(m);
        if (prev >= 0) (void)hipSetDevice(prev);
    }

    // run_copy_inputs_mat_to_hostmem (async.cpp:32-56), restricted to the mappers' source footprint: the
    // rows and columns no kernel of any mapper reads are neither copied nor uploaded
    void copy_in(Job& j) {
        int s = -1;
        if (!free_slots.pop(s)) throw OctvrError(OCTVR_E_INVALID, "pipeline closed");
        j.slot = s;
        stage(j, [&] {
            uint8_t* const dst = slots[s].packed_host->p;
            copy_in_pool.run(runs.size(), [&](size_t lo, size_t hi) {
                for (size_t k = lo; k < hi; k++) {
                    const FootRun& r = runs[k];
                    const int i = (int)(r.cam & 31u), rp = (int)(r.cam >> 8), w = in_w[i];
                    const int x0 = 8 * (int)r.g0, yb = std::min(8 * (int)(r.g0 + r.ng), w) - x0;
                    const int c0 = 4 * (int)r.g0, cb = std::max(0, std::min(4 * (int)(r.g0 + r.ng), w / 2) - c0);
                    const size_t py = j.in_pitches[3 * i], pu = j.in_pitches[3 * i + 1], pv = j.in_pitches[3 * i + 2];
                    uint8_t* d = dst + r.off;
                    memcpy(d, j.in_planes[3 * i] + (size_t)(2 * rp) * py + x0, yb);
                    memcpy(d + yb, j.in_planes[3 * i] + (size_t)(2 * rp + 1) * py + x0, yb);
                    memcpy(d + 2 * yb, j.in_planes[3 * i + 1] + (size_t)rp * pu + c0, cb);
                    memcpy(d + 2 * yb + cb, j.in_planes[3 * i + 2] + (size_t)rp * pv + c0, cb);
                }
            });
        });
    }

    // run_upload_inputs_hostmem_to_gpumat (async.cpp:58-68): the packed runs, then one kernel puts them in
    // place in the device frames (bytes outside the footprint keep whatever they held: nothing reads them)
    void upload(Job& j) {
        stage(j, [&] {
            DeviceGuard dg(device);
            Slot& sl = slots[j.slot];
            if (packed_bytes) {
                HIP_CHECK(hipMemcpyAsync(sl.packed_dev.p, sl.packed_host->p, packed_bytes, hipMemcpyHostToDevice, up));
                HIP_CHECK(launch_unpack_runs(sl.packed_dev.p, runs_dev.p, (int)runs.size(), sl.frames, up));
            }
            HIP_CHECK(hipStreamSynchronize(up));
        });
    }

    // run_do_mapping (async.cpp:70-91)
    void map(Job& j) {
        stage(j, [&] {
            DeviceGuard dg(device);
            Slot& sl = slots[j.slot];
            std::vector<const uint8_t*> in(n_in);
            std::vector<size_t> pitch(n_in);
            for (int i = 0; i < n_in; i++) {
                in[i] = sl.in_dev[i].p;
                pitch[i] = (size_t)in_w[i];
            }
            for (size_t k = 0; k < mappers.size(); k++) {
                const int gm = gain_modes[k];
                const double* chained = nullptr;
                if (gm >= 0 && gm < (int)k && mapper_has_gain(mappers[gm])) chained = mapper_gains_dev(mappers[gm]);
                // preview_output(_rect_mul_size(output_regions[i], preview_output.size())) (async.cpp:75-76): the
                // region's view of the preview image (an empty view is no preview, mapper.cpp:308)
                PreviewOut pv{};
                const bool with_pv = preview_w > 0 && preview_rects[k].w > 0 && preview_rects[k].h > 0;
                if (with_pv) {
                    const Rect& r = preview_rects[k];
                    const size_t pp = (size_t)preview_w * 3;
                    pv = PreviewOut{sl.preview_dev.p + (size_t)r.y * pp + (size_t)r.x * 3, r.w, r.h, pp};
                }
                mapper_stitch(mappers[k], in.data(), pitch.data(), sl.out_dev[k].p, (size_t)regions[k].w, nullptr, 0,
                              chained, comp, with_pv ? &pv : nullptr);
            }
            HIP_CHECK(hipStreamSynchronize(comp));
        });
    }

    // run_download_outputs_gpumat_to_hostmem (async.cpp:93-111)
    void download(Job& j) {
        stage(j, [&] {
            DeviceGuard dg(device);
            Slot& sl = slots[j.slot];
            for (size_t k = 0; k < mappers.size(); k++) {
                if (!j.direct) {
                    HIP_CHECK(hipMemcpyAsync(sl.out_host[k]->p, sl.out_dev[k].p, sl.out_host[k]->n, hipMemcpyDeviceToHost,
                                             down));
                    continue;
                }
                // straight into the caller's registered planes: the region's Y rows, then its chroma rows'
                // U (left) and V (right) halves (the device region is "Y over [U|V]", pitch = region width)
                const Rect& r = regions[k];
                const Rect& c = regions_uv[k];
                const uint8_t* src = sl.out_dev[k].p;
                HIP_CHECK(hipMemcpy2DAsync(j.out_planes[0] + (size_t)r.y * j.out_pitches[0] + r.x, j.out_pitches[0], src,
                                           (size_t)r.w, (size_t)r.w, (size_t)r.h, hipMemcpyDeviceToHost, down));
                HIP_CHECK(hipMemcpy2DAsync(j.out_planes[1] + (size_t)c.y * j.out_pitches[1] + c.x, j.out_pitches[1],
                                           src + (size_t)r.h * r.w, (size_t)r.w, (size_t)c.w, (size_t)c.h,
                                           hipMemcpyDeviceToHost, down));
                HIP_CHECK(hipMemcpy2DAsync(j.out_planes[2] + (size_t)c.y * j.out_pitches[2] + c.x, j.out_pitches[2],
                                           src + (size_t)r.h * r.w + r.w / 2, (size_t)r.w, (size_t)c.w, (size_t)c.h,
                                           hipMemcpyDeviceToHost, down));
            }
            if (preview_w > 0)  // async.cpp:102-103
                HIP_CHECK(hipMemcpyAsync(sl.preview_host->p, sl.preview_dev.p, sl.preview_host->n, hipMemcpyDeviceToHost,
                                         down));
            HIP_CHECK(hipStreamSynchronize(down));
        });
    }

    // run_copy_outputs_hostmem_to_mat (async.cpp:113-172)
    void copy_out(Job& j) {
        stage(j, [&] {
            if (j.direct) return;  // the D2H wrote the caller's planes
            Slot& sl = slots[j.slot];
            for (size_t k = 0; k < mappers.size(); k++) {
                const Rect& r = regions[k];
                const Rect& c = regions_uv[k];
                const uint8_t* src = sl.out_host[k]->p;
                copy_out_pool.run((size_t)(r.h + c.h), [&](size_t lo, size_t hi) {
                    for (size_t y = lo; y < hi; y++) {
                        if (y < (size_t)r.h) {
                            memcpy(j.out_planes[0] + (size_t)(r.y + (int)y) * j.out_pitches[0] + r.x, src + y * r.w, r.w);
                        } else {
                            const size_t cy = y - (size_t)r.h;
                            const uint8_t* row = src + (size_t)(r.h + (int)cy) * r.w;
                            memcpy(j.out_planes[1] + (size_t)(c.y + (int)cy) * j.out_pitches[1] + c.x, row, c.w);
                            memcpy(j.out_planes[2] + (size_t)(c.y + (int)cy) * j.out_pitches[2] + c.x, row + r.w / 2, c.w);
                        }
                    }
                });
            }
        });
        // frame_total_time += fps_timer.tick(); fps over every block of 10 frames (async.cpp:141-147)
        const auto now = std::chrono::steady_clock::now();
        frame_total_ms += std::chrono::duration<double, std::milli>(now - fps_t).count();
        fps_t = now;
        if (++frame_count == 10) {
            frame_fps = 1.0 / (frame_total_ms / (double)frame_count / 1000);
            frame_count = 0;
            frame_total_ms = 0;
        }
        // the preview with its PreviewDataHeader (async.cpp:149-171): published, then handed to the sink
        if (preview_w > 0 && j.status == OCTVR_OK) {
            const Slot& sl = slots[j.slot];
            const octvr_preview_header h{preview_w, preview_h, 0, frame_fps};
            std::lock_guard<std::mutex> g(pub_mu);
            memcpy(pub.data(), sl.preview_host->p, pub.size());
            pub_hdr = h;
            if (sink) sink(sink_user, sl.preview_host->p, (size_t)preview_w * 3, &h);
        }
    }

    template <class F>
    void worker(Channel<std::shared_ptr<Job>>& in, Channel<std::shared_ptr<Job>>& out, F f) {
        std::shared_ptr<Job> j;
        while (in.pop(j)) {
            f(*j);
            out.push(std::move(j));
        }
        out.close();
    }

    void start() {
        threads.emplace_back([this] {
            std::shared_ptr<Job> j;
            while (q_in.pop(j)) {
                try {
                    copy_in(*j);
                } catch (const OctvrError& e) {
                    j->status = e.code;
                    j->error = e.what();
                }
                q_up.push(std::move(j));
            }
            q_up.close();
        });
        threads.emplace_back([this] { worker(q_up, q_map, [this](Job& j) { upload(j); }); });
        threads.emplace_back([this] { worker(q_map, q_down, [this](Job& j) { map(j); }); });
        threads.emplace_back([this] { worker(q_down, q_out, [this](Job& j) { download(j); }); });
        threads.emplace_back([this] {
            std::shared_ptr<Job> j;
            while (q_out.pop(j)) {
                copy_out(*j);
                if (j->slot >= 0) free_slots.push(j->slot);
                q_done.push(std::move(j));
            }
            free_slots.close();
            q_done.close();
        });
    }
};

extern "C" {

int octvr_async_create(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                       const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                       const double* output_regions, octvr_async** out) {
    return octvr_async_create_ex(rigs, n_rigs, device, n_inputs, in_w, in_h, out_w, out_h, blend_modes, gain_modes,
                                 output_regions, 0, out);
}

int octvr_async_create_ex(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                          const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                          const double* output_regions, int flags, octvr_async** out) {
    return octvr_async_create_preview(rigs, n_rigs, device, n_inputs, in_w, in_h, out_w, out_h, blend_modes, gain_modes,
                                      output_regions, flags, 0, 0, out);
}

int octvr_async_create_preview(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                               const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                               const double* output_regions, int flags, int preview_w, int preview_h,
                               octvr_async** out) {
    try {
        REQUIRE(rigs && n_rigs > 0 && in_w && in_h && blend_modes && gain_modes && output_regions && out,
                "NULL argument");
        REQUIRE(n_inputs > 0 && n_inputs <= kMaxCams && out_w > 0 && out_h > 0 && out_w % 2 == 0 && out_h % 2 == 0, "bad sizes");
        REQUIRE(preview_w >= 0 && preview_h >= 0 && (uint64_t)preview_w * (uint64_t)preview_h * 3 < 0x7FFFFF80ull,
                "bad preview size");
        auto a = std::make_unique<octvr_async>();
        a->device = device;
        a->flags = flags;
        // preview_size.area() > 0 enables the preview (async.cpp:99, 299)
        if ((int64_t)preview_w * preview_h > 0) {
            a->preview_w = preview_w;
            a->preview_h = preview_h;
            a->pub.assign((size_t)preview_w * preview_h * 3, 0);
        }
        a->n_in = n_inputs;
        a->out_w = out_w;
        a->out_h = out_h;
        a->in_w.assign(in_w, in_w + n_inputs);
        a->in_h.assign(in_h, in_h + n_inputs);
        a->gain_modes.assign(gain_modes, gain_modes + n_rigs);
        for (int i = 0; i < n_inputs; i++)
            REQUIRE(in_w[i] > 0 && in_h[i] > 0 && in_w[i] % 2 == 0 && in_h[i] % 2 == 0, "input sizes must be even");
        for (int k = 0; k < n_rigs; k++) {
            REQUIRE(rigs[k], "NULL rig");
            const Rect r = rect_mul_size(output_regions + 4 * k, out_w, out_h);
            const Rect c = rect_mul_size(output_regions + 4 * k, out_w / 2, out_h / 2);
            REQUIRE(r.x >= 0 && r.y >= 0 && r.w > 0 && r.h > 0 && r.w % 2 == 0 && r.h % 2 == 0,
                    "output region must be a non-empty even-sized rectangle inside the output");
            // the reference copies the mapper's U / V planes into the region of the output's U / V planes
            // (async.cpp:133-135); a size mismatch would reallocate the destination instead
            REQUIRE(c.w == r.w / 2 && c.h == r.h / 2, "output region's chroma rectangle is not half its luma rectangle");
            a->regions.push_back(r);
            a->regions_uv.push_back(c);
            a->preview_rects.push_back(a->preview_w ? rect_mul_size(output_regions + 4 * k, a->preview_w, a->preview_h)
                                                    : Rect{0, 0, 0, 0});
            octvr_mapper* m = nullptr;
            // Mapper(mts[i], in_sizes, blend_modes[i], gain_modes[i] >= 0, r.size()) (async.cpp:250-255)
            const int rc = octvr_mapper_create_ex(rigs[k], device, n_inputs, in_w, in_h, blend_modes[k],
                                                  gain_modes[k] >= 0 ? 1 : 0, r.w, r.h, flags, &m);
            if (rc != OCTVR_OK) throw OctvrError(rc, std::string("mapper ") + std::to_string(k) + ": " + octvr_last_error());
            a->mappers.push_back(m);
            REQUIRE(mapper_num_inputs(m) == n_inputs, "every rig must have n_inputs inputs (no overlays)");
        }
        DeviceGuard dg(device);
        HIP_CHECK(hipStreamCreateWithFlags(&a->up, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&a->comp, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&a->down, hipStreamNonBlocking));
        // what the mappers read of the inputs: one packed upload of those bytes per frame
        SourceFootprint foot;
        foot.init(a->in_w, a->in_h);
        for (auto* m : a->mappers) foot.merge(mapper_footprint(m));
        a->runs = footprint_runs(foot, a->packed_bytes);
        REQUIRE(a->packed_bytes < ((size_t)1 << 32), "input footprint exceeds 4 GiB");
        if (!a->runs.empty()) a->runs_dev.upload(a->runs.data(), a->runs.size());
        for (auto& sl : a->slots) {
            sl.packed_host.reset(new PinnedBuf());
            sl.packed_host->alloc(std::max<size_t>(a->packed_bytes, 1));
            sl.packed_dev.alloc(std::max<size_t>(a->packed_bytes, 1));
            for (int i = 0; i < n_inputs; i++) {
                const size_t bytes = (size_t)in_w[i] * (in_h[i] / 2 * 3);
                sl.in_dev.emplace_back();
                sl.in_dev.back().alloc(bytes);
                // bytes outside the footprint are never read; a fixed pattern rather than stale memory
                HIP_CHECK(hipMemset(sl.in_dev.back().p, 0x5A, bytes));
                sl.frames.f[i] = sl.in_dev.back().p;
                sl.frames.w[i] = in_w[i];
                sl.frames.h[i] = in_h[i];
            }
            if (a->preview_w) {  // GpuMat(preview_size, CV_8UC3).setTo(0) + HostMem (async.cpp:299-305)
                const size_t pb = (size_t)a->preview_w * a->preview_h * 3;
                sl.preview_dev.alloc(pb);
                HIP_CHECK(hipMemset(sl.preview_dev.p, 0, pb));
                sl.preview_host.reset(new PinnedBuf());
                sl.preview_host->alloc(pb);
            }
            for (int k = 0; k < n_rigs; k++) {
                const size_t bytes = (size_t)a->regions[k].w * (a->regions[k].h / 2 * 3);
                sl.out_host.emplace_back(new PinnedBuf());
                sl.out_host.back()->alloc(bytes);
                sl.out_dev.emplace_back();
                sl.out_dev.back().alloc(bytes);
            }
        }
        for (int s = 0; s < kSlots; s++) a->free_slots.push(s);
        a->start();
        *out = a.release();
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return OCTVR_E_HIP;
    }
}

int octvr_async_push(octvr_async* a, const uint8_t* const* in_planes, const size_t* in_pitches,
                     uint8_t* const* out_planes, const size_t* out_pitches) {
    if (!a || !in_planes || !in_pitches || !out_planes || !out_pitches) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    auto j = std::make_shared<Job>();
    j->in_planes.assign(in_planes, in_planes + 3 * a->n_in);
    j->in_pitches.assign(in_pitches, in_pitches + 3 * a->n_in);
    for (int i = 0; i < a->n_in; i++)
        if (!in_planes[3 * i] || !in_planes[3 * i + 1] || !in_planes[3 * i + 2] || in_pitches[3 * i] < (size_t)a->in_w[i] ||
            in_pitches[3 * i + 1] < (size_t)a->in_w[i] / 2 || in_pitches[3 * i + 2] < (size_t)a->in_w[i] / 2) {
            set_last_error("bad input plane");
            return OCTVR_E_INVALID;
        }
    for (int k = 0; k < 3; k++) {
        j->out_planes[k] = out_planes[k];
        j->out_pitches[k] = out_pitches[k];
        if (!out_planes[k] || out_pitches[k] < (size_t)(k ? a->out_w / 2 : a->out_w)) {
            set_last_error("bad output plane");
            return OCTVR_E_INVALID;
        }
    }
    for (const octvr_async::RegOut& r : a->reg_out)
        j->direct |= r.p[0] == out_planes[0] && r.p[1] == out_planes[1] && r.p[2] == out_planes[2] &&
                     r.pitch[0] == out_pitches[0] && r.pitch[1] == out_pitches[1] && r.pitch[2] == out_pitches[2];
    a->q_in.push(std::move(j));
    a->pending++;
    return OCTVR_OK;
}

int octvr_async_pop(octvr_async* a) {
    if (!a || a->pending <= 0) {
        set_last_error("no frame pending");
        return OCTVR_E_INVALID;
    }
    std::shared_ptr<Job> j;
    if (!a->q_done.pop(j)) {
        set_last_error("pipeline closed");
        return OCTVR_E_INVALID;
    }
    a->pending--;
    if (j->status != OCTVR_OK) set_last_error(j->error);
    return j->status;
}

int octvr_async_pending(const octvr_async* a, int* n) {
    if (!a || !n) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    *n = a->pending;
    return OCTVR_OK;
}

int octvr_async_register_output(octvr_async* a, uint8_t* const* planes, const size_t* pitches) {
    if (!a || !planes || !pitches) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    for (int k = 0; k < 3; k++)
        if (!planes[k] || pitches[k] < (size_t)(k ? a->out_w / 2 : a->out_w)) {
            set_last_error("bad output plane");
            return OCTVR_E_INVALID;
        }
    for (const octvr_async::RegOut& r : a->reg_out)
        if (r.p[0] == planes[0] && r.p[1] == planes[1] && r.p[2] == planes[2] && r.pitch[0] == pitches[0] &&
            r.pitch[1] == pitches[1] && r.pitch[2] == pitches[2])
            return OCTVR_OK;  // already registered
    try {
        DeviceGuard dg(a->device);
        octvr_async::RegOut r{};
        int done = 0;
        for (; done < 3; done++) {
            const size_t rows = done ? (size_t)a->out_h / 2 : (size_t)a->out_h;
            const size_t w = done ? (size_t)a->out_w / 2 : (size_t)a->out_w;
            const hipError_t e = hipHostRegister(planes[done], pitches[done] * (rows - 1) + w, hipHostRegisterDefault);
            if (e != hipSuccess) {
                for (int k = 0; k < done; k++) (void)hipHostUnregister(planes[k]);
                (void)hipGetLastError();
                set_last_error(std::string("hipHostRegister: ") + hipGetErrorString(e));
                return OCTVR_E_HIP;
            }
            r.p[done] = planes[done];
            r.pitch[done] = pitches[done];
        }
        a->reg_out.push_back(r);
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    }
}

int octvr_async_unregister_output(octvr_async* a, uint8_t* const* planes) {
    if (!a || !planes) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    if (a->pending > 0) {  // a queued frame may still be written into them
        set_last_error("frames pending: pop them before unregistering their planes");
        return OCTVR_E_INVALID;
    }
    for (size_t i = 0; i < a->reg_out.size(); i++) {
        const octvr_async::RegOut& r = a->reg_out[i];
        if (r.p[0] != planes[0] || r.p[1] != planes[1] || r.p[2] != planes[2]) continue;
        DeviceGuard dg(a->device);
        for (uint8_t* p : r.p) (void)hipHostUnregister(p);
        a->reg_out.erase(a->reg_out.begin() + (long)i);
        return OCTVR_OK;
    }
    set_last_error("planes not registered");
    return OCTVR_E_INVALID;
}

int octvr_async_pop_preview(octvr_async* a, uint8_t* rgb, size_t pitch, octvr_preview_header* hdr) {
    if (!a || !hdr || (a->preview_w > 0 && (!rgb || pitch < (size_t)a->preview_w * 3))) {
        set_last_error("bad arguments");
        return OCTVR_E_INVALID;
    }
    if (a->preview_w == 0) {
        set_last_error("the pipeline has no preview (preview size 0)");
        return OCTVR_E_INVALID;
    }
    std::lock_guard<std::mutex> g(a->pub_mu);
    *hdr = a->pub_hdr;
    if (a->pub_hdr.width == 0) return OCTVR_OK;  // nothing published yet
    const size_t rb = (size_t)a->preview_w * 3;
    for (int y = 0; y < a->preview_h; y++) memcpy(rgb + (size_t)y * pitch, a->pub.data() + (size_t)y * rb, rb);
    return OCTVR_OK;
}

int octvr_async_set_preview_sink(octvr_async* a, octvr_preview_sink sink, void* user) {
    if (!a) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    std::lock_guard<std::mutex> g(a->pub_mu);
    a->sink = sink;
    a->sink_user = user;
    return OCTVR_OK;
}

int octvr_async_info(const octvr_async* a, char* buf, size_t len) {
    if (!a || !buf || len == 0) {
        set_last_error("bad arguments");
        return OCTVR_E_INVALID;
    }
    size_t in_bytes = 0, out_bytes = 0;
    for (int i = 0; i < a->n_in; i++) in_bytes += (size_t)a->in_w[i] * (a->in_h[i] / 2 * 3);
    for (const Rect& r : a->regions) out_bytes += (size_t)r.w * (r.h / 2 * 3);
    char tmp[512];
    snprintf(tmp, sizeof tmp,
             "{\"mappers\": %d, \"inputs\": %d, \"packed_bytes\": %zu, \"runs\": %zu, \"input_frame_bytes\": %zu, "
             "\"output_bytes\": %zu, \"preview\": [%d, %d], \"flags\": %d, \"slots\": %d}",
             (int)a->mappers.size(), a->n_in, a->packed_bytes, a->runs.size(), in_bytes, out_bytes, a->preview_w,
             a->preview_h, a->flags, kSlots);
    if (strlen(tmp) >= len) {
        set_last_error("buffer too small");
        return OCTVR_E_INVALID;
    }
    memcpy(buf, tmp, strlen(tmp) + 1);
    return OCTVR_OK;
}

void octvr_async_destroy(octvr_async* a) { delete a; }

}  // extern "C"
