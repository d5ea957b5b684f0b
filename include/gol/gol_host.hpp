// gol_host.hpp -- native (C++17) host mirror of the reference's F# grid/generation interface, on top of
// the C ABI (gol.h).  The reference is compiled .NET code; this is its compiled-language counterpart,
// header-only, with the same names, argument meanings and error behaviour as the F# it mirrors:
//
//   Grid, Location, UpdateView, applyGrid   GameOfLife/GameOfLife/GameOfLifeLogic.fs:5-35
//   UpdateAgent (render agent)              GameOfLifeUI.fs:13-35 (GameofLife.fs:42-64): Reset starts a new
//                                           dictionary, each Update inserts, a full dictionary fills the Gray8
//                                           pixels[x + y*size] (128 / 0) and hands over the frame
//   Board                                   replaces the W*H cell agents (GameOfLifeLogic.fs:39-71)
//   run() -> GameOfLife (IDisposable)       GameOfLifeDriver.fs:13-41: seeded board, updateView = one tick =
//                                           UpdateView.Reset + one generation + the W*H Update posts (or one
//                                           rendered frame), optional timer (L38-40)
//
// Errors: the F# code fails with exceptions (failwith); every failing C-ABI call here throws gol::Error
// carrying gol_last_error().  The reference has no error channel for its agents.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "gol.h"

namespace gol {

struct Error : std::runtime_error {
    int code;
    Error(const std::string& what, int c) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* what) {
    if (rc != GOL_OK) throw Error(std::string(what) + " failed (" + std::to_string(rc) + "): " + gol_last_error(), rc);
}

// ---------------------------------------------------------------- GameOfLifeLogic.fs:5-35
constexpr int size = 100;                        // L5
struct Grid {                                    // L6
    int Width;
    int Height;
};
constexpr Grid grid{size, size};                 // L8
constexpr int gridProduct = size * size;         // L7
struct Location {                                // L10-11 ([<Struct>] {x; y})
    int x;
    int y;
    bool operator<(const Location& o) const { return x != o.x ? x < o.x : y < o.y; }
    bool operator==(const Location& o) const { return x == o.x && y == o.y; }
};
struct UpdateView {                              // L32-35: Reset | Update of bool * Location
    enum Kind { Reset, Update } kind;
    bool alive = false;
    Location location{0, 0};
    static UpdateView reset() { return {Reset, false, {0, 0}}; }
    static UpdateView update(bool a, Location l) { return {Update, a, l}; }
};
template <class F>
void applyGrid(F&& f, Grid g = grid) {           // L13-15: x outer, y inner
    for (int x = 0; x < g.Width; x++)
        for (int y = 0; y < g.Height; y++) f(x, y);
}

// ---------------------------------------------------------------- the board (replaces the cell agents)
class Board {
   public:
    // num_gpus > 1: row strips over devices 0..num_gpus-1 of this process (gol.h gol_create)
    Board(int64_t width, int64_t height, int boundary = GOL_TORUS, int tblock_k = 0, int num_gpus = 1)
        : w_(width), h_(height) {
        check(gol_create(width, height, boundary, num_gpus, tblock_k, &b_), "gol_create");
    }
    // explicit strip placement (gol_create_multi), e.g. {0, 0} runs two strips on one GPU
    Board(int64_t width, int64_t height, int boundary, int tblock_k, const std::vector<int>& devices)
        : w_(width), h_(height) {
        check(gol_create_multi(width, height, boundary, devices.data(), (int)devices.size(), tblock_k, 0, &b_),
              "gol_create_multi");
    }
    ~Board() {
        if (b_) gol_destroy(b_);
    }
    Board(const Board&) = delete;
    Board& operator=(const Board&) = delete;
    Board(Board&& o) noexcept : b_(std::exchange(o.b_, nullptr)), w_(o.w_), h_(o.h_) {}

    int64_t width() const { return w_; }
    int64_t height() const { return h_; }
    Board& seedDotnet(int32_t seed, int mode = GOL_INIT_DOTNET_MOD2) {
        check(gol_seed_dotnet(b_, seed, mode), "gol_seed_dotnet");
        return *this;
    }
    Board& setCells(const std::vector<uint8_t>& cells) {
        check(gol_set_cells(b_, cells.data(), (int64_t)cells.size()), "gol_set_cells");
        return *this;
    }
    Board& placeRle(const std::string& rle, int64_t x, int64_t y) {
        check(gol_place_rle(b_, rle.c_str(), x, y), "gol_place_rle");
        return *this;
    }
    Board& step(int64_t generations = 1) {
        check(gol_step(b_, generations), "gol_step");
        return *this;
    }
    std::vector<uint8_t> getCells() const {  // cells[x + y*W]
        std::vector<uint8_t> c((size_t)(w_ * h_));
        check(gol_get_cells(b_, c.data(), (int64_t)c.size()), "gol_get_cells");
        return c;
    }
    std::vector<uint8_t> renderGray8(uint8_t alive_value = 128) const {
        std::vector<uint8_t> p((size_t)(w_ * h_));
        check(gol_render_gray8(b_, p.data(), w_, alive_value), "gol_render_gray8");
        return p;
    }
    int64_t generation() const {
        int64_t g = 0;
        check(gol_generation(b_, &g), "gol_generation");
        return g;
    }
    int64_t population() const {
        int64_t p = 0;
        check(gol_population(b_, &p), "gol_population");
        return p;
    }
    uint64_t hash() const {
        uint64_t h = 0;
        check(gol_hash(b_, &h), "gol_hash");
        return h;
    }
    gol_board* handle() const { return b_; }

   private:
    gol_board* b_ = nullptr;
    int64_t w_, h_;
};

// ---------------------------------------------------------------- GameOfLifeUI.fs:13-35 (headless)
class UpdateAgent {
   public:
    using FrameFn = std::function<void(const std::vector<uint8_t>&)>;
    explicit UpdateAgent(Grid g = grid, uint8_t alive_value = 128, FrameFn on_frame = nullptr)
        : grid_(g), alive_(alive_value), pixels_((size_t)g.Width * g.Height, 0), on_frame_(std::move(on_frame)) {}

    void post(const UpdateView& msg) {
        std::lock_guard<std::mutex> lk(mu_);
        if (msg.kind == UpdateView::Reset) {  // L20: a new Dictionary
            states_.clear();
            return;
        }
        states_[msg.location] = msg.alive;  // L22
        if ((int64_t)states_.size() == (int64_t)grid_.Width * grid_.Height) {  // L23
            for (const auto& kv : states_)  // L24-28: pixels[x + y*size]
                pixels_[(size_t)(kv.first.x + kv.first.y * grid_.Width)] = kv.second ? alive_ : 0;
            frame_locked();
        }
    }
    // fast path: one frame rendered on the GPU instead of W*H Update messages
    void postFrame(std::vector<uint8_t> pixels) {
        std::lock_guard<std::mutex> lk(mu_);
        pixels_ = std::move(pixels);
        frame_locked();
    }
    int64_t frames() const { return frames_; }
    uint8_t aliveValue() const { return alive_; }
    Grid gridSize() const { return grid_; }
    std::vector<uint8_t> pixels() const {
        std::lock_guard<std::mutex> lk(mu_);
        return pixels_;
    }

   private:
    void frame_locked() {  // L29-31: WritePixels on the UI thread
        frames_++;
        if (on_frame_) on_frame_(pixels_);
    }
    Grid grid_;
    uint8_t alive_;
    std::vector<uint8_t> pixels_;
    FrameFn on_frame_;
    std::map<Location, bool> states_;  // Dictionary(HashIdentity.Structural)
    mutable std::mutex mu_;
    std::atomic<int64_t> frames_{0};
};

// ---------------------------------------------------------------- GameOfLifeDriver.fs:13-41
class GameOfLife {  // what run() returns: IDisposable
   public:
    enum class Emit { Updates, Pixels };
    GameOfLife(Board board, UpdateAgent& agent, Emit emit) : board_(std::move(board)), agent_(agent), emit_(emit) {}
    ~GameOfLife() { Dispose(); }
    GameOfLife(const GameOfLife&) = delete;
    GameOfLife& operator=(const GameOfLife&) = delete;

    // L32-34: one tick = UpdateView.Reset, then one generation for every cell.  Ticks may re-enter from
    // the timer (L38-40): serialised here.
    void updateView() {
        std::lock_guard<std::mutex> lk(tick_);
        agent_.post(UpdateView::reset());
        board_.step(1);
        if (emit_ == Emit::Pixels) {
            agent_.postFrame(board_.renderGray8(agent_.aliveValue()));
            return;
        }
        const auto cells = board_.getCells();
        const Grid g = agent_.gridSize();
        applyGrid([&](int x, int y) { agent_.post(UpdateView::update(cells[(size_t)(x + y * g.Width)] != 0, {x, y})); },
                  g);
    }
    // L38-40: a timer calling updateView every period.  A failed tick stops the timer and is kept for
    // lastError() (an exception escaping the thread would terminate the process; the .NET timer handler of
    // the reference does not bring the process down either).
    void start(std::chrono::milliseconds period) {
        timer_ = std::thread([this, period] {
            std::unique_lock<std::mutex> lk(stop_mu_);
            while (!stop_cv_.wait_for(lk, period, [this] { return stop_; })) {
                lk.unlock();
                try {
                    updateView();
                } catch (...) {
                    lk.lock();
                    error_ = std::current_exception();
                    stop_ = true;
                    break;
                }
                lk.lock();
            }
        });
    }
    // the exception of the tick that stopped the timer, or nullptr
    std::exception_ptr lastError() {
        std::lock_guard<std::mutex> lk(stop_mu_);
        return error_;
    }
    void Dispose() {
        {
            std::lock_guard<std::mutex> lk(stop_mu_);
            stop_ = true;
        }
        stop_cv_.notify_all();
        if (timer_.joinable()) timer_.join();
    }
    Board& board() { return board_; }

   private:
    Board board_;
    UpdateAgent& agent_;
    Emit emit_;
    std::mutex tick_;
    std::thread timer_;
    std::exception_ptr error_;
    std::mutex stop_mu_;
    std::condition_variable stop_cv_;
    bool stop_ = false;
};

// L13-41.  `seed` replaces `int DateTime.Now.Ticks` (L10) so runs are reproducible; the board is seeded
// x outer / y inner with Random.Next() % 2 = 0 (L9-11,16-19).  period 0 = no timer (ticks by hand).
inline GameOfLife* run(UpdateAgent& agent, int32_t seed, int boundary = GOL_TORUS,
                       std::chrono::milliseconds period = std::chrono::milliseconds(0),
                       GameOfLife::Emit emit = GameOfLife::Emit::Updates, int tblock_k = 0) {
    const Grid g = agent.gridSize();
    Board b(g.Width, g.Height, boundary, tblock_k);
    b.seedDotnet(seed, GOL_INIT_DOTNET_MOD2);
    auto* game = new GameOfLife(std::move(b), agent, emit);
    if (period.count() > 0) game->start(period);
    return game;
}

}  // namespace gol
