// gol_multi.h -- one board handle over several GPUs of one process (gol_create with num_gpus > 1,
// gol_create_multi).  Not installed; gol_capi.cpp dispatches the public entry points here.
//
// Halo transport (gol_set_option "transport", include/gol/gol.h): peer copies (hipMemcpyPeerAsync over xGMI, or a
// device-local copy when a device repeats) by default; RCCL (ncclSend / ncclRecv inside ncclGroupStart / End, one
// communicator per part from ncclCommInitAll over the parts' devices) on request when every part has its own device
// -- RCCL refuses two ranks on one GPU.  The default stays on peer copies until a parity test has run the RCCL
// transport on distinct GPUs; bench.py's handle leg runs both and compares their hashes.  Both follow
// the same plan (exchange_plan), checked on the CPU by tests/test_exchange_order.py.
//
// The reference's host is ONE process (the F# driver, GameOfLifeDriver.fs:13-41), so a drop-in that
// spreads the board over the GPUs of a node must do it behind one handle.  Layout: row strips, part r
// owning global rows [y0_r, y0_r + rows_r) on devices[r], in the gol_strip geometry of include/gol/gol.h
// (ghost = tblock halo rows above and below).  Per pass of k generations each part sends its top and
// bottom k owned rows into its neighbours' ghost rows on a copy stream, while its interior rows [k, rows-k) run on
// the compute stream; the two k-row edge bands run on an edge stream once the ghost rows have landed.  The result is
// bit-identical to the single board.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/gol/gol.h"

namespace gol {

int api_fail(int code, const std::string& msg);  // sets gol_last_error (gol_capi.cpp)
// gol_strip_step / gol_strip_plan with a board's streaming options ("split", "seg_rows", "seam", "split2";
// gol_capi.cpp)
int strip_step_opts(const gol_strip* s, const uint32_t* src, uint32_t* dst, int k, int64_t out_begin, int64_t out_end,
                    hipStream_t stream, int32_t split_opt, int64_t seg_opt, int32_t seam_opt, int32_t split2_opt = 0);
int strip_plan_opts(const gol_strip* s, int k, int64_t out_begin, int64_t out_end, int64_t* waves, int64_t* seg_rows,
                    int32_t split_opt, int64_t seg_opt, int32_t seam_opt, int32_t split2_opt = 0);

// The halo messages of one pass, in the order each part issues them (include/gol/gol.h gol_xfer): part r sends its
// top k owned rows to `up` and its bottom k rows to `down`, then receives the down neighbour's top rows below its
// owned rows and the up neighbour's bottom rows above them.  RCCL pairs a sender's sends to one peer with that
// peer's receives from it in issue order (tags are ignored), which this order satisfies even when up == down (two
// parts on a torus).  Rows are buffer rows (0 = the first of `ghost` halo rows above the owned rows).
std::vector<gol_xfer> exchange_plan(int64_t height, int boundary, int nparts, int64_t ghost, int k);

class MultiBoard {
   public:
    struct Part {
        int device = 0;
        gol_strip s{};
        uint32_t* buf[2] = {nullptr, nullptr};
        unsigned long long* acc = nullptr;
        hipStream_t compute = nullptr, edge = nullptr, copy = nullptr;
        hipEvent_t ev_start = nullptr, ev_copied = nullptr, ev_edge = nullptr;
        int up = -1, down = -1;  // neighbour parts (-1: bounded board edge)
        void* comm = nullptr;    // ncclComm_t of this part (RCCL transport)
    };

    // creates the parts; returns GOL_OK or a GOL_ERR_* code (the object is then unusable)
    int init(int64_t width, int64_t height, int boundary, const int* devices, int n, int tblock, int ilv);
    ~MultiBoard();

    int set_cells(const uint8_t* host);
    int readback(uint8_t* host, int64_t stride, uint8_t value);
    int region(int64_t x, int64_t y, int64_t w, int64_t h, uint8_t* out);
    int seed_splitmix(uint64_t seed);
    int save_packed(uint64_t* host);        // canonical snapshot rows (gol_save_packed)
    int load_packed(const uint64_t* host);
    int clear();
    int place_points(const std::vector<int64_t>& xy);  // global (x, y) pairs, already wrapped
    int step(int64_t generations, int64_t* done);      // *done: generations actually advanced
    // step() between HIP events on every part's compute stream; *elapsed_us = the longest part's span (gol_step_timed)
    int step_timed(int64_t generations, int64_t* done, double* elapsed_us);
    int reduce(bool hash, uint64_t* out);
    int synchronize();
    // one pass of the board's depth with timing events (gol_pass_timing): per part, microseconds from the
    // pass start to the interior launch's end, to the edge stream's release (halo copies landed) and to the
    // edge bands' end
    int timed_pass(double* interior_us, double* wait_us, double* edge_us, int64_t* done);

    // halo transport: GOL_TRANSPORT_PEER (default) or GOL_TRANSPORT_RCCL (creates the communicators on first use;
    // GOL_ERR_UNSUPPORTED when a device repeats or RCCL is unavailable, and the board keeps its transport)
    int set_transport(int transport);
    // streaming-pass options of the board (gol_set_option "split", "seg_rows", "seam", "split2"), applied to every
    // strip launch
    void set_stream_options(int32_t split_opt, int64_t seg_opt, int32_t seam_opt, int32_t split2_opt) {
        split_opt_ = split_opt;
        seg_opt_ = seg_opt;
        seam_opt_ = seam_opt;
        split2_opt_ = split2_opt;
    }

    int parts() const { return (int)parts_.size(); }
    const Part& part(int i) const { return parts_[(size_t)i]; }
    int cur() const { return cur_; }
    hipStream_t stream0() const { return parts_.empty() ? nullptr : parts_[0].compute; }
    int max_k() const { return max_k_; }
    int transport() const { return rccl_ ? GOL_TRANSPORT_RCCL : GOL_TRANSPORT_PEER; }
    const std::string& transport_note() const { return transport_note_; }

   private:
    struct PassTimer {  // timing events of one part, recorded only by timed_pass
        hipEvent_t t0 = nullptr, interior = nullptr, go = nullptr, edge = nullptr;
    };
    int pass(int k, std::vector<PassTimer>* timers = nullptr);
    int exchange_peer(int k);
    int exchange_rccl(int k);
    int init_rccl();
    int strip_step(const gol_strip& s, const uint32_t* src, uint32_t* dst, int k, int64_t b, int64_t e,
                   hipStream_t st) const;
    std::vector<Part> parts_;
    bool rccl_ = false;       // the transport in use
    bool comms_ = false;      // RCCL communicators exist (parts_[i].comm)
    bool distinct_ = false;   // every part has its own device
    int32_t split_opt_ = 0, seam_opt_ = 0, split2_opt_ = 0;
    int64_t seg_opt_ = 0;
    std::string transport_note_;
    int64_t W_ = 0, H_ = 0;
    int boundary_ = GOL_TORUS, ilv_ = 1, tblock_ = 1, max_k_ = 1;
    int cur_ = 0;
};

}  // namespace gol
