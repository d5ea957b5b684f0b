// gol_multi.cpp -- a board handle spread over several GPUs of one process (see gol_multi.h).
//
// Replaces, for a board too large or too slow for one GPU, the same reference seam as the single board:
// the dictionary of cell actors built by GameOfLifeDriver.fs:16-30 and ticked by updateView (L32-34).
// The per-pass protocol (ghost rows of depth k, interior || exchange, then the edge bands) is the one the
// one-process-per-GPU path runs over torch.distributed (strips.py).  Here one process drives every part: the
// exchange is a peer copy ordered by HIP events (the default), or on request (gol_set_option "transport") RCCL
// send/recv over a communicator spanning the parts' devices (ncclCommInitAll) when every part has its own GPU.
#include "gol_multi.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>

#include "gol_internal.h"

namespace gol {

#define GOL_MHIP(expr)                                                                                    \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) return api_fail(GOL_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define GOL_MRC(expr)              \
    do {                           \
        int rc_ = (expr);          \
        if (rc_ != GOL_OK) return rc_; \
    } while (0)

namespace {

// device staging buffer freed on every exit path
struct Staging {
    void* p = nullptr;
    ~Staging() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t n) {
        hipError_t e = hipMalloc(&p, n ? n : 1);
        if (e != hipSuccess) {
            p = nullptr;
            return api_fail(GOL_ERR_OOM, std::string("hipMalloc staging: ") + hipGetErrorString(e));
        }
        return GOL_OK;
    }
};

// RCCL, resolved at run time (dlopen): a process that never builds a multi-GPU board does not need librccl, and a
// process that already loaded one (torch bundles its own under the same soname) shares it instead of loading a
// second copy.
struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;  // why it is unavailable

    static const Rccl& get() {
        static const Rccl r = [] {
            Rccl x;
            void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) {
                const char* e = dlerror();
                x.error = std::string("dlopen librccl.so.1: ") + (e ? e : "?");
                return x;
            }
            x.init_all = (decltype(x.init_all))dlsym(h, "ncclCommInitAll");
            x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
            x.send = (decltype(x.send))dlsym(h, "ncclSend");
            x.recv = (decltype(x.recv))dlsym(h, "ncclRecv");
            x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
            x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
            x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
            if (!x.init_all || !x.destroy || !x.send || !x.recv || !x.group_start || !x.group_end || !x.error_string)
                x.error = "librccl.so.1 lacks a symbol of the send/recv API";
            return x;
        }();
        return r;
    }
    bool ok() const { return error.empty(); }
    std::string why(ncclResult_t r) const { return error_string ? error_string(r) : "rccl error"; }
};

}  // namespace

std::vector<gol_xfer> exchange_plan(int64_t height, int boundary, int nparts, int64_t ghost, int k) {
    std::vector<gol_xfer> ops;
    const bool torus = boundary == GOL_TORUS;
    for (int r = 0; r < nparts; r++) {
        const int64_t rows = height * (r + 1) / nparts - height * r / nparts;
        const int up = r > 0 ? r - 1 : (torus ? nparts - 1 : -1);
        const int down = r < nparts - 1 ? r + 1 : (torus ? 0 : -1);
        auto add = [&](int op, int peer, int64_t row) { ops.push_back(gol_xfer{r, op, peer, 0, row, k}); };
        if (up >= 0) add(0, up, ghost);                        // my top k owned rows -> up's bottom ghost
        if (down >= 0) add(0, down, ghost + rows - k);         // my bottom k owned rows -> down's top ghost
        if (down >= 0) add(1, down, ghost + rows);             // down's top rows -> my bottom ghost
        if (up >= 0) add(1, up, ghost - k);                    // up's bottom rows -> my top ghost
    }
    return ops;
}

// Creates the RCCL communicators (once); GOL_ERR_UNSUPPORTED with the reason when RCCL cannot serve this board.
int MultiBoard::init_rccl() {
    if (comms_) return GOL_OK;
    if (!distinct_) return api_fail(GOL_ERR_UNSUPPORTED, "RCCL transport: a device holds more than one part (RCCL needs "
                                                         "one rank per GPU)");
    const Rccl& nc = Rccl::get();
    if (!nc.ok()) return api_fail(GOL_ERR_UNSUPPORTED, "RCCL transport: " + nc.error);
    std::vector<int> devs;
    for (const Part& p : parts_) devs.push_back(p.device);
    std::vector<ncclComm_t> comms(parts_.size(), nullptr);
    const ncclResult_t r = nc.init_all(comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) return api_fail(GOL_ERR_UNSUPPORTED, "RCCL transport: ncclCommInitAll failed: " + nc.why(r));
    for (size_t i = 0; i < parts_.size(); i++) parts_[i].comm = comms[i];
    comms_ = true;
    return GOL_OK;
}

int MultiBoard::set_transport(int transport) {
    if (transport != GOL_TRANSPORT_PEER && transport != GOL_TRANSPORT_RCCL)
        return api_fail(GOL_ERR_INVALID, "transport must be 1 (peer copies) or 2 (RCCL)");
    GOL_MRC(synchronize());  // no pass of the old transport is in flight
    if (transport == GOL_TRANSPORT_RCCL) {
        GOL_MRC(init_rccl());
        rccl_ = true;
        transport_note_ = "RCCL ncclSend/ncclRecv over one communicator per part (ncclCommInitAll, " +
                          std::to_string(parts_.size()) + " devices)";
    } else {
        rccl_ = false;
        transport_note_ = distinct_ ? "peer copies: hipMemcpyPeerAsync between the parts' devices (the default)"
                                    : "peer copies: a device holds more than one part (RCCL needs one rank per GPU)";
    }
    return GOL_OK;
}

// gol_strip_step with the board's streaming options (gol_capi.cpp)
int MultiBoard::strip_step(const gol_strip& s, const uint32_t* src, uint32_t* dst, int k, int64_t b, int64_t e,
                           hipStream_t st) const {
    return strip_step_opts(&s, src, dst, k, b, e, st, split_opt_, seg_opt_, seam_opt_, split2_opt_);
}

int MultiBoard::init(int64_t width, int64_t height, int boundary, const int* devices, int n, int tblock, int ilv) {
    W_ = width;
    H_ = height;
    boundary_ = boundary;
    ilv_ = ilv;
    tblock_ = tblock;
    if (n < 2 || !devices) return api_fail(GOL_ERR_INVALID, "a multi-GPU board needs at least 2 parts");
    if (height < n) return api_fail(GOL_ERR_INVALID, "fewer board rows than GPUs");
    // balanced row partition: part r owns [H*r/n, H*(r+1)/n)
    int64_t min_rows = height;
    for (int r = 0; r < n; r++) min_rows = std::min(min_rows, height * (r + 1) / n - height * r / n);
    // a pass of k generations reads k ghost rows on each side, which come from ONE neighbour strip
    max_k_ = stream_largest_k(std::min<int64_t>(tblock, min_rows), tblock, ilv, width / 32, boundary == GOL_BOUNDED);
    parts_.resize((size_t)n);
    for (int r = 0; r < n; r++) {
        Part& p = parts_[(size_t)r];
        p.device = devices[r];
        p.s.width = width;
        p.s.height = height;
        p.s.y0 = height * r / n;
        p.s.rows = height * (r + 1) / n - p.s.y0;
        p.s.ghost = max_k_;
        p.s.pitch = width / 32;
        p.s.boundary = boundary;
        p.s.wrap_rows = 0;
        p.s.ilv = ilv;
        p.s.spare_waves = 0;
        const bool torus = boundary == GOL_TORUS;
        p.up = r > 0 ? r - 1 : (torus ? n - 1 : -1);
        p.down = r < n - 1 ? r + 1 : (torus ? 0 : -1);
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipStreamCreateWithFlags(&p.compute, hipStreamNonBlocking));
        GOL_MHIP(hipStreamCreateWithFlags(&p.edge, hipStreamNonBlocking));
        GOL_MHIP(hipStreamCreateWithFlags(&p.copy, hipStreamNonBlocking));
        GOL_MHIP(hipEventCreateWithFlags(&p.ev_start, hipEventDisableTiming));
        GOL_MHIP(hipEventCreateWithFlags(&p.ev_copied, hipEventDisableTiming));
        GOL_MHIP(hipEventCreateWithFlags(&p.ev_edge, hipEventDisableTiming));
        const size_t bytes = (size_t)((p.s.rows + 2 * p.s.ghost) * p.s.pitch) * 4;
        for (auto& b : p.buf) {
            hipError_t e = hipMalloc(&b, bytes);
            if (e != hipSuccess) {
                b = nullptr;
                return api_fail(GOL_ERR_OOM, std::string("hipMalloc strip: ") + hipGetErrorString(e));
            }
            GOL_MHIP(hipMemsetAsync(b, 0, bytes, p.compute));
        }
        GOL_MHIP(hipMalloc(&p.acc, 64));
    }
    // peer copies by default; RCCL on request (set_transport) when every part has its own device
    std::vector<int> seen;
    distinct_ = true;
    for (const Part& p : parts_) {
        if (std::find(seen.begin(), seen.end(), p.device) != seen.end()) distinct_ = false;
        seen.push_back(p.device);
    }
    rccl_ = false;
    transport_note_ = distinct_ ? "peer copies: hipMemcpyPeerAsync between the parts' devices (the default)"
                                : "peer copies: a device holds more than one part (RCCL needs one rank per GPU)";
    // peer access between neighbouring parts on distinct devices (xGMI); without it the copies are staged
    for (const Part& p : parts_)
        for (int q : {p.up, p.down}) {
            if (q < 0 || parts_[(size_t)q].device == p.device) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, p.device, parts_[(size_t)q].device) == hipSuccess && can) {
                GOL_MHIP(hipSetDevice(p.device));
                hipError_t e = hipDeviceEnablePeerAccess(parts_[(size_t)q].device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return api_fail(GOL_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();
            }
        }
    return synchronize();
}

MultiBoard::~MultiBoard() {
    for (Part& p : parts_) {
        if (hipSetDevice(p.device) != hipSuccess) continue;
        for (hipStream_t s : {p.compute, p.edge, p.copy})
            if (s) (void)hipStreamSynchronize(s);
        if (p.comm) (void)Rccl::get().destroy(static_cast<ncclComm_t>(p.comm));
        for (auto b : p.buf)
            if (b) (void)hipFree(b);
        if (p.acc) (void)hipFree(p.acc);
        for (hipEvent_t e : {p.ev_start, p.ev_copied, p.ev_edge})
            if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : {p.compute, p.edge, p.copy})
            if (s) (void)hipStreamDestroy(s);
    }
}

int MultiBoard::synchronize() {
    for (const Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipStreamSynchronize(p.copy));
        GOL_MHIP(hipStreamSynchronize(p.edge));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::set_cells(const uint8_t* host) {
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        const size_t n = (size_t)(p.s.rows * W_);
        Staging st;
        GOL_MRC(st.alloc(n));
        GOL_MHIP(hipMemcpyAsync(st.p, host + p.s.y0 * W_, n, hipMemcpyHostToDevice, p.compute));
        GOL_MRC(gol_strip_pack(&p.s, static_cast<const uint8_t*>(st.p), p.buf[cur_], p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::readback(uint8_t* host, int64_t stride, uint8_t value) {
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        const size_t n = (size_t)(p.s.rows * stride);
        Staging st;
        GOL_MRC(st.alloc(n));
        if (stride != W_) GOL_MHIP(hipMemsetAsync(st.p, 0, n, p.compute));
        GOL_MRC(gol_strip_unpack(&p.s, p.buf[cur_], static_cast<uint8_t*>(st.p), stride, value, p.compute));
        GOL_MHIP(hipMemcpyAsync(host + p.s.y0 * stride, st.p, n, hipMemcpyDeviceToHost, p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::region(int64_t x, int64_t y, int64_t w, int64_t h, uint8_t* out) {
    for (Part& p : parts_) {
        const int64_t r0 = std::max(y, p.s.y0), r1 = std::min(y + h, p.s.y0 + p.s.rows);
        if (r0 >= r1) continue;
        GOL_MHIP(hipSetDevice(p.device));
        const size_t n = (size_t)((r1 - r0) * w);
        Staging st;
        GOL_MRC(st.alloc(n));
        GOL_MHIP(launch_region(p.buf[cur_] + p.s.ghost * p.s.pitch, ilv_, W_, p.s.pitch, x, r0 - p.s.y0, w, r1 - r0,
                               static_cast<uint8_t*>(st.p), p.compute));
        GOL_MHIP(hipMemcpyAsync(out + (r0 - y) * w, st.p, n, hipMemcpyDeviceToHost, p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::save_packed(uint64_t* host) {
    const int64_t nc = (W_ + 63) / 64;
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        const size_t n = (size_t)(p.s.rows * nc) * 8;
        Staging st;
        GOL_MRC(st.alloc(n));
        GOL_MHIP(launch_export_canonical(p.buf[cur_], W_, p.s.rows, p.s.pitch, p.s.ghost, ilv_,
                                         static_cast<uint64_t*>(st.p), p.compute));
        GOL_MHIP(hipMemcpyAsync(host + p.s.y0 * nc, st.p, n, hipMemcpyDeviceToHost, p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::load_packed(const uint64_t* host) {
    const int64_t nc = (W_ + 63) / 64;
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        const size_t n = (size_t)(p.s.rows * nc) * 8;
        Staging st;
        GOL_MRC(st.alloc(n));
        GOL_MHIP(hipMemcpyAsync(st.p, host + p.s.y0 * nc, n, hipMemcpyHostToDevice, p.compute));
        GOL_MHIP(launch_import_canonical(static_cast<const uint64_t*>(st.p), W_, p.s.rows, p.s.pitch, p.s.ghost, ilv_,
                                         p.buf[cur_], p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::seed_splitmix(uint64_t seed) {
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MRC(gol_strip_seed_splitmix(&p.s, p.buf[cur_], seed, p.compute));
    }
    return synchronize();
}

int MultiBoard::clear() {
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        const size_t bytes = (size_t)((p.s.rows + 2 * p.s.ghost) * p.s.pitch) * 4;
        GOL_MHIP(hipMemsetAsync(p.buf[cur_], 0, bytes, p.compute));
    }
    return synchronize();
}

int MultiBoard::place_points(const std::vector<int64_t>& xy) {
    for (Part& p : parts_) {
        std::vector<int64_t> mine;
        for (size_t i = 0; i + 1 < xy.size(); i += 2)
            if (xy[i + 1] >= p.s.y0 && xy[i + 1] < p.s.y0 + p.s.rows) {
                mine.push_back(xy[i]);
                mine.push_back(xy[i + 1] - p.s.y0);  // owned row
            }
        if (mine.empty()) continue;
        GOL_MHIP(hipSetDevice(p.device));
        Staging st;
        GOL_MRC(st.alloc(mine.size() * sizeof(int64_t)));
        GOL_MHIP(hipMemcpyAsync(st.p, mine.data(), mine.size() * sizeof(int64_t), hipMemcpyHostToDevice, p.compute));
        GOL_MHIP(launch_set_points(p.buf[cur_] + p.s.ghost * p.s.pitch, ilv_, W_, p.s.pitch,
                                   static_cast<const int64_t*>(st.p), (int64_t)mine.size() / 2, p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
    }
    return GOL_OK;
}

int MultiBoard::reduce(bool hash, uint64_t* out) {
    uint64_t sum = 0;
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipMemsetAsync(p.acc, 0, sizeof(unsigned long long), p.compute));
        uint64_t* acc = reinterpret_cast<uint64_t*>(p.acc);
        GOL_MRC(hash ? gol_strip_hash_partial(&p.s, p.buf[cur_], acc, p.compute)
                     : gol_strip_population(&p.s, p.buf[cur_], acc, p.compute));
        unsigned long long v = 0;
        GOL_MHIP(hipMemcpyAsync(&v, p.acc, sizeof(v), hipMemcpyDeviceToHost, p.compute));
        GOL_MHIP(hipStreamSynchronize(p.compute));
        sum += (uint64_t)v;  // hash partials add with wrap-around
    }
    *out = hash ? gol_hash_finalize(sum, W_, H_) : sum;
    return GOL_OK;
}

// One pass of k generations over every part (the ordering argument is in DESIGN.md 5):
//   compute[i]: record ev_start (previous pass of part i complete: compute joined edge at its end)
//   copy[i]:    wait ev_start[i]; top k owned rows -> up's bottom ghost, bottom k -> down's top ghost;
//               record ev_copied[i]
//   compute[i]: interior rows [k, rows-k) (needs no ghost rows, overlaps the copies)
//   edge[i]:    wait ev_start[i], ev_copied[up], ev_copied[down]; rows [0, k) and [rows-k, rows)
//   compute[i]: wait ev_edge[i]
// A copy into part j's ghost rows is ordered after j's previous pass has read them: the copying part's
// previous pass waited for j's copies, which waited for j's pass before that.
// Peer copies: each part pushes its edge rows into its neighbours' ghost rows on its copy stream (after its own
// previous pass); a part's edge bands then wait for its NEIGHBOURS' copy streams.
int MultiBoard::exchange_peer(int k) {
    const size_t row_bytes = (size_t)W_ / 8;  // pitch == width / 32 words
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipStreamWaitEvent(p.copy, p.ev_start, 0));
        const uint32_t* src = p.buf[cur_];
        if (p.up >= 0) {
            Part& u = parts_[(size_t)p.up];
            GOL_MHIP(hipMemcpyPeerAsync(u.buf[cur_] + (u.s.ghost + u.s.rows) * u.s.pitch, u.device,
                                        src + p.s.ghost * p.s.pitch, p.device, k * row_bytes, p.copy));
        }
        if (p.down >= 0) {
            Part& d = parts_[(size_t)p.down];
            GOL_MHIP(hipMemcpyPeerAsync(d.buf[cur_] + (d.s.ghost - k) * d.s.pitch, d.device,
                                        src + (p.s.ghost + p.s.rows - k) * p.s.pitch, p.device, k * row_bytes,
                                        p.copy));
        }
        GOL_MHIP(hipEventRecord(p.ev_copied, p.copy));
    }
    return GOL_OK;
}

// RCCL: every part's sends and receives of the pass in ONE group (one thread drives every communicator), issued
// in exchange_plan's order on each part's copy stream after that part's previous pass; a part's edge bands then
// wait for its OWN copy stream, where its receives complete.
int MultiBoard::exchange_rccl(int k) {
    const Rccl& nc = Rccl::get();
    const std::vector<gol_xfer> plan = exchange_plan(H_, boundary_, (int)parts_.size(), max_k_, k);
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipStreamWaitEvent(p.copy, p.ev_start, 0));
    }
    ncclResult_t r = nc.group_start();
    if (r != ncclSuccess) return api_fail(GOL_ERR_HIP, "ncclGroupStart: " + nc.why(r));
    for (const gol_xfer& x : plan) {
        Part& p = parts_[(size_t)x.part];
        uint32_t* rows = p.buf[cur_] + x.row * p.s.pitch;
        const size_t bytes = (size_t)(x.nrows * p.s.pitch) * 4;
        r = x.op == 0 ? nc.send(rows, bytes, ncclUint8, x.peer, static_cast<ncclComm_t>(p.comm), p.copy)
                      : nc.recv(rows, bytes, ncclUint8, x.peer, static_cast<ncclComm_t>(p.comm), p.copy);
        if (r != ncclSuccess) {
            (void)nc.group_end();
            return api_fail(GOL_ERR_HIP, std::string(x.op == 0 ? "ncclSend: " : "ncclRecv: ") + nc.why(r));
        }
    }
    r = nc.group_end();
    if (r != ncclSuccess) return api_fail(GOL_ERR_HIP, "ncclGroupEnd: " + nc.why(r));
    for (Part& p : parts_) {
        GOL_MHIP(hipSetDevice(p.device));
        GOL_MHIP(hipEventRecord(p.ev_copied, p.copy));
    }
    return GOL_OK;
}

int MultiBoard::pass(int k, std::vector<PassTimer>* timers) {
    for (size_t i = 0; i < parts_.size(); i++) {
        Part& p = parts_[i];
        GOL_MHIP(hipSetDevice(p.device));
        if (timers) GOL_MHIP(hipEventRecord((*timers)[i].t0, p.compute));
        GOL_MHIP(hipEventRecord(p.ev_start, p.compute));
    }
    GOL_MRC(rccl_ ? exchange_rccl(k) : exchange_peer(k));
    for (size_t i = 0; i < parts_.size(); i++) {
        Part& p = parts_[i];
        GOL_MHIP(hipSetDevice(p.device));
        const uint32_t* src = p.buf[cur_];
        uint32_t* dst = p.buf[cur_ ^ 1];
        const int64_t rows = p.s.rows;
        const int64_t lo = std::min<int64_t>(k, rows), hi = std::max<int64_t>(rows - k, lo);
        if (lo < hi) {
            // leave room on the device for the two edge bands, which start as soon as the ghost rows land
            int64_t w0 = 0, w1 = 0;
            GOL_MRC(strip_plan_opts(&p.s, k, 0, lo, &w0, nullptr, split_opt_, seg_opt_, seam_opt_, split2_opt_));
            GOL_MRC(strip_plan_opts(&p.s, k, hi, rows, &w1, nullptr, split_opt_, seg_opt_, seam_opt_, split2_opt_));
            gol_strip s = p.s;
            s.spare_waves = (int32_t)std::min<int64_t>(w0 + w1, 1 << 20);
            GOL_MRC(strip_step(s, src, dst, k, lo, hi, p.compute));
        }
        if (timers) GOL_MHIP(hipEventRecord((*timers)[i].interior, p.compute));
        GOL_MHIP(hipStreamWaitEvent(p.edge, p.ev_start, 0));
        if (rccl_) {
            GOL_MHIP(hipStreamWaitEvent(p.edge, p.ev_copied, 0));  // my receives landed
        } else {
            for (int q : {p.up, p.down})
                if (q >= 0) GOL_MHIP(hipStreamWaitEvent(p.edge, parts_[(size_t)q].ev_copied, 0));
        }
        if (timers) GOL_MHIP(hipEventRecord((*timers)[i].go, p.edge));
        GOL_MRC(strip_step(p.s, src, dst, k, 0, lo, p.edge));
        GOL_MRC(strip_step(p.s, src, dst, k, hi, rows, p.edge));
        if (timers) GOL_MHIP(hipEventRecord((*timers)[i].edge, p.edge));
        GOL_MHIP(hipEventRecord(p.ev_edge, p.edge));
        GOL_MHIP(hipStreamWaitEvent(p.compute, p.ev_edge, 0));
    }
    cur_ ^= 1;
    return GOL_OK;
}

int MultiBoard::timed_pass(double* interior_us, double* wait_us, double* edge_us, int64_t* done) {
    std::vector<PassTimer> t(parts_.size());
    auto destroy = [&t, this]() {
        for (size_t i = 0; i < t.size(); i++) {
            (void)hipSetDevice(parts_[i].device);
            for (hipEvent_t e : {t[i].t0, t[i].interior, t[i].go, t[i].edge})
                if (e) (void)hipEventDestroy(e);
        }
    };
    int rc = GOL_OK;
    for (size_t i = 0; i < t.size() && rc == GOL_OK; i++) {
        if (hipSetDevice(parts_[i].device) != hipSuccess) rc = api_fail(GOL_ERR_HIP, "hipSetDevice");
        for (hipEvent_t* e : {&t[i].t0, &t[i].interior, &t[i].go, &t[i].edge})
            if (rc == GOL_OK && hipEventCreate(e) != hipSuccess) rc = api_fail(GOL_ERR_HIP, "hipEventCreate");
    }
    if (rc == GOL_OK) rc = pass(max_k_, &t);
    if (rc == GOL_OK) rc = synchronize();
    for (size_t i = 0; i < t.size() && rc == GOL_OK; i++) {
        float a = 0, b = 0, c = 0;
        if (hipSetDevice(parts_[i].device) != hipSuccess || hipEventElapsedTime(&a, t[i].t0, t[i].interior) != hipSuccess ||
            hipEventElapsedTime(&b, t[i].t0, t[i].go) != hipSuccess ||
            hipEventElapsedTime(&c, t[i].t0, t[i].edge) != hipSuccess) {
            rc = api_fail(GOL_ERR_HIP, "hipEventElapsedTime");
            break;
        }
        interior_us[i] = 1e3 * a;
        wait_us[i] = 1e3 * b;
        edge_us[i] = 1e3 * c;
    }
    if (rc == GOL_OK) *done += max_k_;
    destroy();
    return rc;
}

int MultiBoard::step_timed(int64_t generations, int64_t* done, double* elapsed_us) {
    // events of one device are only comparable with each other: each part times its own span (first to last
    // launch of the call on its compute stream, which joins its edge stream at the end of every pass)
    std::vector<hipEvent_t> ev(2 * parts_.size(), nullptr);
    int rc = GOL_OK;
    for (size_t i = 0; i < parts_.size() && rc == GOL_OK; i++) {
        if (hipSetDevice(parts_[i].device) != hipSuccess || hipEventCreate(&ev[2 * i]) != hipSuccess ||
            hipEventCreate(&ev[2 * i + 1]) != hipSuccess || hipEventRecord(ev[2 * i], parts_[i].compute) != hipSuccess)
            rc = api_fail(GOL_ERR_HIP, "step timing: event setup failed");
    }
    if (rc == GOL_OK) rc = step(generations, done);
    double worst = 0;
    for (size_t i = 0; i < parts_.size() && rc == GOL_OK; i++) {
        float ms = 0;
        if (hipSetDevice(parts_[i].device) != hipSuccess || hipEventRecord(ev[2 * i + 1], parts_[i].compute) != hipSuccess ||
            hipEventSynchronize(ev[2 * i + 1]) != hipSuccess || hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) != hipSuccess)
            rc = api_fail(GOL_ERR_HIP, "step timing: event readout failed");
        worst = std::max(worst, 1e3 * (double)ms);
    }
    for (size_t i = 0; i < parts_.size(); i++) {
        (void)hipSetDevice(parts_[i].device);
        for (int j = 0; j < 2; j++)
            if (ev[2 * i + j]) (void)hipEventDestroy(ev[2 * i + j]);
    }
    if (rc == GOL_OK) {
        rc = synchronize();
        *elapsed_us = worst;
    }
    return rc;
}

int MultiBoard::step(int64_t generations, int64_t* done) {
    while (generations > 0) {
        const int k = stream_largest_k(generations, max_k_, ilv_, W_ / 32, boundary_ == GOL_BOUNDED);
        GOL_MRC(pass(k));
        generations -= k;
        *done += k;
    }
    return GOL_OK;
}

}  // namespace gol
