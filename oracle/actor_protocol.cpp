// actor_protocol.cpp -- CPU restatement of the reference's per-cell ACTOR protocol.
// TEST INFRASTRUCTURE / CPU BASELINE ONLY ("cpu_baseline.kind = port" in bench.py).  Never linked
// into the product library.
//
// What it restates (message for message):
//   cell actor        GameOfLife/GameOfLife/GameOfLifeLogic.fs:39-71  (Akka twin GameofLife.fs:88-138)
//     Reset          L47-52: send State(self) to the 8 neighbours, Clear neighbourStates, wasAlive <- isAlive
//     State(c)       L54:    c (NeighbourState(location, wasAlive))
//     NeighbourState L56-66: neighbourStates.[cell] <- alive; when Count = 8 apply the rule (L59-63),
//                           post Update(alive, location) to the update agent, isAlive <- next
//   update agent      GameOfLifeUI.fs:13-35: Reset starts a new Dictionary; each Update inserts; when
//                     Count = gridProduct the Gray8 pixels are filled (128 / 0, index x + y*size)
//   driver            GameOfLifeDriver.fs:13-41: cells created x outer / y inner with Random.Next()%2=0,
//                     torus neighbour lists (dx outer, dy inner, skip self) L21-25, wiring L27-30,
//                     updateView L32-34 = post UpdateView.Reset, then Reset to every cell.
//
// Transport: one FIFO mailbox per actor (MailboxProcessor / Akka UnboundedMailbox), actors scheduled
// on a pool of worker threads with an Akka-like throughput of 30 messages per turn.
//
// Determinism: the reference fans Reset out while cells already run (AsParallel().ForAll,
// GameOfLifeDriver.fs:34), so a State request can overtake a neighbour's Reset.
// This restatement applies the Reset->State PHASE BARRIER that defines parity: every Reset is enqueued
// before any actor runs in a generation, so each mailbox's FIFO delivers its Reset before any State.
// Under that barrier the protocol equals the synchronous double-buffered step of gol_oracle.c; the
// test suite checks that equality.  A generation ends when the update agent has rendered the frame
// (its Dictionary reached gridProduct entries).
//
// Without the barrier (SURVEY.md section 8f, rank 4 -- demonstration only, never a parity reference):
// SCHEDULE "racy-seq:S" replays one schedule the reference permits, deterministically on one thread:
// the driver posts Reset to the cells in a shuffled order (seed S), and every message that Reset causes
// is delivered before the next Reset is posted.  A State request then reaches the cells not yet reset in
// this generation, which answer with their stale wasAlive (GameOfLifeLogic.fs:54 reads wasAlive, set only
// by Reset, L52) -- the reference's race, made reproducible.  Different S give different boards.
//
// Usage: actor_protocol W H GENS THREADS SEED [MIN_SECONDS] [INIT] [SCHEDULE]
//   INIT = "dotnet-mod2" (default; GameOfLifeDriver.fs:9-11) or "splitmix"
//   SCHEDULE = "barrier" (default) or "racy-seq:S"
//   Runs GENS generations, or as many as needed to reach MIN_SECONDS of wall time when GENS <= 0.
//   Prints one JSON line: generations, seconds, cell_updates_per_s, messages, hash, population.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

extern "C" {
int oracle_seed_dotnet(uint8_t* cells, int64_t W, int64_t H, int32_t seed, int mode);
int oracle_seed_splitmix(uint8_t* cells, int64_t W, int64_t H, uint64_t seed);
uint64_t oracle_hash(const uint8_t* cells, int64_t W, int64_t H);
int64_t oracle_population(const uint8_t* cells, int64_t W, int64_t H);
}

namespace {

enum Kind : uint8_t { kReset = 0, kState = 1, kNeighbourState = 2, kUpdate = 3, kViewReset = 4 };

struct Msg {
    Kind kind;
    uint8_t alive;
    int32_t who;  // State: reply-to actor; NeighbourState / Update: sender location index
};

struct Actor {
    std::mutex mu;
    std::deque<Msg> box;
    bool scheduled = false;
};

struct CellState {  // GameOfLifeLogic.fs:24-30 `State` + the per-cell Dictionary (L40)
    int32_t neighbours[8];
    bool was_alive = false;
    bool is_alive = false;
    int32_t ns_keys[8];
    uint8_t ns_vals[8];
    int ns_count = 0;
};

class System {
   public:
    System(int64_t W, int64_t H, int threads, const uint8_t* init)
        : W_(W), H_(H), n_(W * H), actors_(n_ + 1), cells_(n_), queues_(threads > 0 ? threads : 1),
          nthreads_(threads) {
        agent_id_ = (int32_t)n_;
        for (int64_t x = 0; x < W; x++)
            for (int64_t y = 0; y < H; y++) {
                CellState& c = cells_[idx(x, y)];
                c.is_alive = init[x + y * W] != 0;  // createDeafault alive (wasAlive = false)
                int k = 0;
                for (int64_t nx = x - 1; nx <= x + 1; nx++)
                    for (int64_t ny = y - 1; ny <= y + 1; ny++)
                        if (nx != x || ny != y) c.neighbours[k++] = idx((nx + W) % W, (ny + H) % H);
            }
        pixels_.assign((size_t)n_, 0);
        for (int t = 0; t < threads; t++) workers_.emplace_back([this, t] { worker(t); });
    }

    ~System() {
        {
            std::lock_guard<std::mutex> g(run_mu_);
            stop_ = true;
        }
        run_cv_.notify_all();
        for (auto& w : workers_) w.join();
    }

    // One generation = one updateView() with the phase barrier, waiting for the frame.
    void generation() {
        frame_done_ = false;
        // UpdateView.Reset first (GameOfLifeDriver.fs:33), then Reset to every cell (L34) --
        // all enqueued before any actor runs (phase barrier).
        enqueue_raw(agent_id_, Msg{kViewReset, 0, -1});
        for (int64_t i = 0; i < n_; i++) enqueue_raw((int32_t)i, Msg{kReset, 0, -1});
        for (int64_t i = 0; i <= n_; i++) {
            actors_[i].scheduled = true;
            queues_[i % nthreads_].push((int32_t)i);
        }
        {
            std::lock_guard<std::mutex> g(done_mu_);
            acks_ = 0;
        }
        {
            std::lock_guard<std::mutex> g(run_mu_);
            epoch_++;
        }
        run_cv_.notify_all();
        // the frame is rendered AND every worker has left this epoch before the next tick starts
        std::unique_lock<std::mutex> lk(done_mu_);
        done_cv_.wait(lk, [this] { return frame_done_.load() && acks_ == nthreads_; });
    }

    // One generation without the phase barrier, on the calling thread (construct with threads = 0):
    // Reset to the cells in the order `perm`, each Reset's message cascade delivered before the next.
    void generation_racy_sequential(const std::vector<int32_t>& perm) {
        uint64_t local = 0;
        frame_done_ = false;
        post(agent_id_, Msg{kViewReset, 0, -1}, 0);
        drain(local);
        for (int32_t id : perm) {
            post(id, Msg{kReset, 0, -1}, 0);
            drain(local);
        }
        messages_.fetch_add(local);
    }

    void snapshot(uint8_t* out) const {
        for (int64_t y = 0; y < H_; y++)
            for (int64_t x = 0; x < W_; x++) out[x + y * W_] = pixels_[x + y * W_] ? 1 : 0;
    }

    uint64_t messages() const { return messages_.load(); }

   private:
    int32_t idx(int64_t x, int64_t y) const { return (int32_t)(x * H_ + y); }  // creation order, x outer

    struct Queue {
        std::mutex mu;
        std::deque<int32_t> q;
        void push(int32_t v) {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(v);
        }
        bool pop(int32_t& v) {
            std::lock_guard<std::mutex> g(mu);
            if (q.empty()) return false;
            v = q.front();
            q.pop_front();
            return true;
        }
    };

    void enqueue_raw(int32_t to, const Msg& m) { actors_[to].box.push_back(m); }

    void drain(uint64_t& nmsg) {
        int32_t id;
        while (queues_[0].pop(id)) run_actor(id, 0, nmsg);
    }

    void post(int32_t to, const Msg& m, int self_q) {
        Actor& a = actors_[to];
        bool sched = false;
        {
            std::lock_guard<std::mutex> g(a.mu);
            a.box.push_back(m);
            if (!a.scheduled) {
                a.scheduled = true;
                sched = true;
            }
        }
        if (sched) queues_[self_q].push(to);
    }

    void worker(int t) {
        uint64_t seen_epoch = 0;
        uint64_t local_msgs = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(run_mu_);
                run_cv_.wait(lk, [&] { return stop_ || epoch_ != seen_epoch; });
                if (stop_) return;
                seen_epoch = epoch_;
            }
            int idle = 0;
            while (!frame_done_.load(std::memory_order_relaxed)) {
                int32_t id;
                bool got = queues_[t].pop(id);
                for (int k = 1; !got && k < nthreads_; k++) got = queues_[(t + k) % nthreads_].pop(id);
                if (!got) {
                    if (++idle > 64) std::this_thread::yield();
                    continue;
                }
                idle = 0;
                run_actor(id, t, local_msgs);
            }
            messages_.fetch_add(local_msgs);
            local_msgs = 0;
            {
                std::lock_guard<std::mutex> g(done_mu_);
                acks_++;
            }
            done_cv_.notify_all();
        }
    }

    void run_actor(int32_t id, int t, uint64_t& nmsg) {
        Actor& a = actors_[id];
        for (int turn = 0; turn < 30; turn++) {  // Akka default dispatcher throughput = 30
            Msg m;
            {
                std::lock_guard<std::mutex> g(a.mu);
                if (a.box.empty()) {
                    a.scheduled = false;
                    return;
                }
                m = a.box.front();
                a.box.pop_front();
            }
            nmsg++;
            if (id == agent_id_)
                agent_receive(m);
            else
                cell_receive(id, m, t);
        }
        // throughput exhausted: yield the actor back to the pool
        bool empty;
        {
            std::lock_guard<std::mutex> g(a.mu);
            empty = a.box.empty();
            if (empty) a.scheduled = false;
        }
        if (!empty) queues_[t].push(id);
    }

    // GameOfLifeLogic.fs:45-66
    void cell_receive(int32_t id, const Msg& m, int t) {
        CellState& c = cells_[id];
        switch (m.kind) {
            case kReset:  // L47-52
                for (int k = 0; k < 8; k++) post(c.neighbours[k], Msg{kState, 0, id}, t);
                c.ns_count = 0;
                c.was_alive = c.is_alive;
                break;
            case kState:  // L54
                post(m.who, Msg{kNeighbourState, (uint8_t)c.was_alive, id}, t);
                break;
            case kNeighbourState: {  // L56-66
                int k = 0;
                while (k < c.ns_count && c.ns_keys[k] != m.who) k++;
                if (k == c.ns_count) {
                    c.ns_keys[k] = m.who;
                    c.ns_count++;
                }
                c.ns_vals[k] = m.alive;
                if (c.ns_count == 8) {
                    int a = 0;
                    for (int j = 0; j < 8; j++) a += c.ns_vals[j];
                    bool next = (a > 3 || a < 2) ? false : (a == 3 ? true : c.is_alive);
                    post(agent_id_, Msg{kUpdate, (uint8_t)next, id}, t);
                    c.is_alive = next;
                }
                break;
            }
            default:
                break;
        }
    }

    // GameOfLifeUI.fs:17-33
    void agent_receive(const Msg& m) {
        if (m.kind == kViewReset) {
            states_.clear();
            states_.reserve((size_t)n_);
            return;
        }
        states_[m.who] = m.alive != 0;
        if ((int64_t)states_.size() == n_) {
            for (int64_t x = 0; x < W_; x++)
                for (int64_t y = 0; y < H_; y++) {
                    auto it = states_.find(idx(x, y));
                    pixels_[x + y * W_] = (it != states_.end() && it->second) ? 128 : 0;
                }
            {
                std::lock_guard<std::mutex> g(done_mu_);
                frame_done_ = true;
            }
            done_cv_.notify_all();
        }
    }

    int64_t W_, H_, n_;
    int32_t agent_id_;
    std::vector<Actor> actors_;
    std::vector<CellState> cells_;
    std::vector<Queue> queues_;
    int nthreads_;
    std::vector<std::thread> workers_;
    std::unordered_map<int32_t, bool> states_;
    std::vector<uint8_t> pixels_;
    std::mutex run_mu_;
    std::condition_variable run_cv_;
    uint64_t epoch_ = 0;
    bool stop_ = false;
    std::mutex done_mu_;
    std::condition_variable done_cv_;
    std::atomic<bool> frame_done_{false};
    int acks_ = 0;
    std::atomic<uint64_t> messages_{0};
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s W H GENS THREADS SEED [MIN_SECONDS] [INIT]\n", argv[0]);
        return 2;
    }
    int64_t W = std::atoll(argv[1]), H = std::atoll(argv[2]), gens = std::atoll(argv[3]);
    int threads = std::atoi(argv[4]);
    long long seed = std::atoll(argv[5]);
    double min_s = argc > 6 ? std::atof(argv[6]) : 0.0;
    std::string init = argc > 7 ? argv[7] : "dotnet-mod2";
    std::string schedule = argc > 8 ? argv[8] : "barrier";
    const bool racy = schedule.rfind("racy-seq:", 0) == 0;
    if (W < 3 || H < 3 || threads < 1 || (!racy && schedule != "barrier")) {
        std::fprintf(stderr, "W, H must be >= 3, THREADS >= 1, SCHEDULE barrier | racy-seq:S\n");
        return 2;
    }
    uint64_t rs = racy ? std::strtoull(schedule.c_str() + 9, nullptr, 10) : 0;
    auto next_rand = [&rs]() {  // splitmix64 stream for the schedule shuffle
        uint64_t z = (rs += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    if (racy) threads = 0;
    std::vector<uint8_t> board((size_t)(W * H));
    if (init == "splitmix")
        oracle_seed_splitmix(board.data(), W, H, (uint64_t)seed);
    else
        oracle_seed_dotnet(board.data(), W, H, (int32_t)seed, 0);

    System sys(W, H, threads, board.data());
    auto t0 = std::chrono::steady_clock::now();
    int64_t done = 0;
    double secs = 0;
    for (;;) {
        if (gens > 0 && done >= gens) break;
        if (gens <= 0 && secs >= min_s && done > 0) break;
        if (racy) {
            std::vector<int32_t> perm((size_t)(W * H));
            for (size_t i = 0; i < perm.size(); i++) perm[i] = (int32_t)i;
            for (size_t i = perm.size() - 1; i > 0; i--) std::swap(perm[i], perm[next_rand() % (i + 1)]);
            sys.generation_racy_sequential(perm);
        } else {
            sys.generation();
        }
        done++;
        secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    sys.snapshot(board.data());
    std::printf(
        "{\"schedule\": \"%s\", \"width\": %lld, \"height\": %lld, \"generations\": %lld, \"threads\": %d, \"seconds\": %.6f, "
        "\"cell_updates_per_s\": %.3f, \"messages\": %llu, \"hash\": %llu, \"population\": %lld}\n",
        schedule.c_str(), (long long)W, (long long)H, (long long)done, threads, secs, (double)(W * H) * done / secs,
        (unsigned long long)sys.messages(), (unsigned long long)oracle_hash(board.data(), W, H),
        (long long)oracle_population(board.data(), W, H));
    return 0;
}
