// Probe (one GPU): how RCCL behaves when rank 1 of a 2-rank communicator never joins.
// mode 0: non-blocking init (ncclCommInitRankConfig, blocking = 0), poll 4 s, then ncclCommAbort.
// mode 1: blocking init on a helper thread, wait 4 s, detach it, then exit.
// mode 2: non-blocking init, poll 4 s, leave the communicator (no abort), then exit.
// Every step prints with a timestamp, so a hang names the call it is in.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

static double now() {
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
#define SAY(...) do { std::printf("[%7.3f] ", now()); std::printf(__VA_ARGS__); std::printf("\n"); std::fflush(stdout); } while (0)

int main(int argc, char **argv) {
    const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
    hipSetDevice(0);
    ncclUniqueId id;
    SAY("mode %d: ncclGetUniqueId -> %d", mode, (int)ncclGetUniqueId(&id));
    if (mode == 1) {
        ncclComm_t c = nullptr;
        volatile bool done = false;
        std::thread t([&] { ncclResult_t r = ncclCommInitRank(&c, 2, id, 0); SAY("blocking init returned %d", (int)r); done = true; });
        for (int i = 0; i < 40 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
        SAY("after 4 s: done=%d; detaching the init thread", (int)done);
        t.detach();
        SAY("returning from main");
        return 0;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&c, 2, id, 0, &cfg);
    SAY("ncclCommInitRankConfig -> %d (comm %p)", (int)r, (void *)c);
    for (int i = 0; i < 40 && r == ncclInProgress; ++i) {
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        ncclResult_t e = ncclCommGetAsyncError(c, &r);
        if (i % 10 == 0) SAY("poll %d: GetAsyncError -> %d, state %d", i, (int)e, (int)r);
    }
    SAY("after polling: state %d", (int)r);
    if (mode == 0) {
        std::thread w([] { for (int i = 0; i < 20; ++i) { std::this_thread::sleep_for(std::chrono::seconds(1)); SAY("  (abort still running)"); } });
        w.detach();
        SAY("ncclCommAbort ...");
        r = ncclCommAbort(c);
        SAY("ncclCommAbort -> %d", (int)r);
    }
    SAY("returning from main");
    return 0;
}
