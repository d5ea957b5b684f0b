// Tests of the native host mirror (include/gol/gol_host.hpp) of the reference's F# driver interface,
// written the way the reference's own driver is used: run() -> updateView() ticks -> the render agent's
// frames.  Checked against the CPU oracle (oracle/gol_oracle.c, linked here as the checker only).
//
//   test_host_driver gpu   -- on an MI355X: frames of run()/updateView() vs the oracle, both emit modes,
//                             the timer, applyGrid order, error behaviour
//   test_host_driver cpu   -- without a GPU: board creation fails loudly (gol::Error, GOL_ERR_NO_DEVICE)
// Prints one JSON line {"checks": n, "failures": [...]}; exit status 0 iff no failure.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gol/gol_host.hpp"

extern "C" {  // the CPU oracle (test infrastructure)
int oracle_seed_dotnet(uint8_t* cells, int64_t W, int64_t H, int32_t seed, int mode);
int oracle_step(const uint8_t* in, uint8_t* out, int64_t W, int64_t H, int boundary);
int oracle_render_gray8(const uint8_t* cells, int64_t W, int64_t H, uint8_t* pixels, int64_t stride, uint8_t value);
}

static int checks = 0;
static std::vector<std::string> failures;
#define CHECK(cond)                                                                   \
    do {                                                                              \
        checks++;                                                                     \
        if (!(cond)) failures.push_back(std::string(#cond) + " @" + std::to_string(__LINE__)); \
    } while (0)

static std::vector<std::vector<uint8_t>> oracle_frames(int w, int h, int32_t seed, int n, uint8_t value) {
    std::vector<uint8_t> a((size_t)(w * h)), b(a.size()), px(a.size());
    oracle_seed_dotnet(a.data(), w, h, seed, GOL_INIT_DOTNET_MOD2);
    std::vector<std::vector<uint8_t>> out;
    for (int i = 0; i < n; i++) {
        oracle_step(a.data(), b.data(), w, h, GOL_TORUS);
        a.swap(b);
        oracle_render_gray8(a.data(), w, h, px.data(), w, value);
        out.push_back(px);
    }
    return out;
}

static void gpu_tests() {
    using namespace gol;
    // applyGrid order: x outer, y inner (GameOfLifeLogic.fs:13-15)
    {
        std::vector<std::pair<int, int>> seen;
        applyGrid([&](int x, int y) { seen.emplace_back(x, y); }, Grid{3, 2});
        CHECK(seen.size() == 6 && seen[0] == std::make_pair(0, 0) && seen[1] == std::make_pair(0, 1) &&
              seen[2] == std::make_pair(1, 0));
    }
    // run() on the reference's default board: three ticks through the Update messages, then the pixel path
    const auto want = oracle_frames(size, size, 42, 3, 128);
    {
        std::vector<std::vector<uint8_t>> frames;
        UpdateAgent agent(grid, 128, [&](const std::vector<uint8_t>& p) { frames.push_back(p); });
        GameOfLife* game = run(agent, 42);
        for (int i = 0; i < 3; i++) game->updateView();
        CHECK(frames.size() == 3);
        for (size_t i = 0; i < frames.size() && i < want.size(); i++) CHECK(frames[i] == want[i]);
        CHECK(game->board().generation() == 3);
        delete game;
    }
    {
        std::vector<std::vector<uint8_t>> frames;
        UpdateAgent agent(grid, 128, [&](const std::vector<uint8_t>& p) { frames.push_back(p); });
        GameOfLife* game = run(agent, 42, GOL_TORUS, std::chrono::milliseconds(0), GameOfLife::Emit::Pixels);
        for (int i = 0; i < 3; i++) game->updateView();
        CHECK(frames.size() == 3 && frames == want);
        delete game;
    }
    // the timer (GameOfLifeDriver.fs:38-40): ticks arrive on their own; Dispose stops them
    {
        UpdateAgent agent(grid);
        GameOfLife* game = run(agent, 7, GOL_TORUS, std::chrono::milliseconds(5));
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
        game->Dispose();
        const int64_t n = agent.frames();
        CHECK(n >= 1);
        CHECK(game->board().generation() == n);
        std::this_thread::sleep_for(std::chrono::milliseconds(30));
        CHECK(agent.frames() == n);  // no tick after Dispose
        delete game;
    }
    // one board over row strips (gol_create_multi): devices {0, 0, 0} here, 0..n-1 on a multi-GPU node
    {
        const int w = 128, h = 96;
        std::vector<uint8_t> a((size_t)(w * h)), b2(a.size()), px(a.size());
        oracle_seed_dotnet(a.data(), w, h, 42, GOL_INIT_DOTNET_MOD2);
        for (int i = 0; i < 20; i++) {
            oracle_step(a.data(), b2.data(), w, h, GOL_TORUS);
            a.swap(b2);
        }
        oracle_render_gray8(a.data(), w, h, px.data(), w, 128);
        Board mb(w, h, GOL_TORUS, 0, std::vector<int>{0, 0, 0});
        mb.seedDotnet(42).step(20);
        CHECK(mb.renderGray8(128) == px);
        CHECK(mb.generation() == 20);
    }
    // error behaviour: invalid geometry throws with the library's code and message
    {
        bool threw = false;
        try {
            Board b(2, 2);
        } catch (const Error& e) {
            threw = e.code == GOL_ERR_INVALID && std::string(e.what()).find("gol_create") != std::string::npos;
        }
        CHECK(threw);
    }
}

static void cpu_tests() {
    bool threw = false;
    try {
        gol::Board b(100, 100);
    } catch (const gol::Error& e) {
        threw = e.code == GOL_ERR_NO_DEVICE;
    }
    CHECK(threw);
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    if (gpu)
        gpu_tests();
    else
        cpu_tests();
    std::printf("{\"mode\": \"%s\", \"checks\": %d, \"failures\": [", gpu ? "gpu" : "cpu", checks);
    for (size_t i = 0; i < failures.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", failures[i].c_str());
    std::printf("]}\n");
    return failures.empty() ? 0 : 1;
}
