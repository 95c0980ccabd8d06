// Host test of ThreadSafeQueue<FmBatch*> (include/dropin/fm_batch.h): the reference's one-slot
// protocol (threadsafequeue.h:24-74) with recycled batches. One producer and two consumers run
// N payloads; every consumer must see every payload once, in order; a batch may only be handed
// out again after both consumers prepared it; with 2 batches the producer never holds more than
// 2 at once. No GPU: the HIP event members are never touched.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "fm_batch.h"

int main() {
    constexpr int N = 20000;
    ThreadSafeQueue<FmBatch*> q;
    std::vector<FmBatch> pool(2);
    std::atomic<int> in_use[2] = {{0}, {0}};   // consumers still reading batch i
    for (auto& b : pool) q.add_free(&b);
    std::atomic<int> errors{0};
    auto consumer = [&](int ind) {
        long long expect = 0;
        for (;;) {
            FmBatch* b = nullptr;
            q.wait_and_pop(b, ind);
            if (!b) break;
            if (b->block != expect) errors++;
            expect++;
            const int idx = (int)(b - pool.data());
            in_use[idx]++;
            std::this_thread::yield();
            in_use[idx]--;
            q.prepare(ind);
        }
        if (expect != N) errors++;
    };
    std::thread c0(consumer, 0), c1(consumer, 1);
    for (long long i = 0; i < N; i++) {
        FmBatch* b = q.acquire();
        const int idx = (int)(b - pool.data());
        if (in_use[idx].load() != 0) errors++;   // handed out while a consumer still reads it
        b->block = i;
        q.push(b);
    }
    q.push(nullptr);
    c0.join();
    c1.join();
    std::printf("{\"payloads\": %d, \"errors\": %d}\n", N, errors.load());
    return errors.load() ? 1 : 0;
}
