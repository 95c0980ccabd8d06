// fm_batch.h -- the device-resident payload of the one-slot queue: instead of the
// reference's heap std::vector<float>* fm_demod block (rffrontend.cpp:55, deleted by the next push,
// threadsafequeue.h:34-36), a multi-channel producer hands its consumers a batch descriptor --
// fm_demod[nch][block_if] in device memory plus HIP events -- and batches are recycled, not
// deleted, once both consumers have called prepare().
//
// The protocol of ThreadSafeQueue (push / wait_and_pop / prepare, include/threadsafequeue.h:24-74)
// is kept; what changes is the ordering of the device work behind it, which stays asynchronous on
// the host:
//   producer:  b = q.acquire()                     a free batch (blocks while both are in use)
//              hipStreamWaitEvent(s, b->released[0..1])  consumers' reads of its previous payload
//              ... write b->d_fm on stream s ...; hipEventRecord(b->ready, s); q.push(b)
//   consumer i: q.wait_and_pop(b, i); hipStreamWaitEvent(s_i, b->ready)
//              ... read b->d_fm on s_i ...; hipEventRecord(b->released[i], s_i); q.prepare(i)
// push(nullptr) ends the stream (consumers pop nullptr and stop).
#ifndef SDR_DROPIN_FM_BATCH_H
#define SDR_DROPIN_FM_BATCH_H

#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstddef>
#include <mutex>
#include <vector>

#include "threadsafequeue.h"

struct FmBatch {
    float* d_fm = nullptr;          // [nch][stride] f32, device
    size_t stride = 0;              // elements between channels
    int nch = 0, n = 0;             // channels, samples per channel (block_if)
    long long block = -1;           // block index of the payload
    hipEvent_t ready = nullptr;     // recorded by the producer after writing d_fm
    hipEvent_t released[2] = {nullptr, nullptr};   // recorded by consumer 0 / 1 after reading it
};

// ThreadSafeQueue<FmBatch*>: the reference's protocol over a pool of recycled device batches
template <>
class ThreadSafeQueue<FmBatch *> {
public:
    ThreadSafeQueue() = default;
    ThreadSafeQueue(const ThreadSafeQueue &) = delete;
    ThreadSafeQueue &operator=(const ThreadSafeQueue &) = delete;

    // batches the producer may fill (their events must be created; `released` recorded at least
    // once or never waited on before the first use)
    void add_free(FmBatch *b) {
        std::lock_guard<std::mutex> lk(m_);
        free_.push_back(b);
        free_cv_.notify_all();
    }

    FmBatch *acquire() {
        std::unique_lock<std::mutex> lk(m_);
        free_cv_.wait(lk, [this] { return !free_.empty(); });
        FmBatch *b = free_.back();
        free_.pop_back();
        return b;
    }

    void push(FmBatch *value) {   // threadsafequeue.h:29-41: waits for both consumers' prepare()
        std::unique_lock<std::mutex> lk(m_);
        free_cv_.wait(lk, [this] { return released_[0] && released_[1]; });
        if (slot_) free_.push_back(slot_);   // recycle instead of delete
        slot_ = value;
        released_[0] = released_[1] = false;
        taken_[0] = taken_[1] = false;
        full_ = true;
        avail_cv_.notify_all();
        free_cv_.notify_all();
    }

    void wait_and_pop(FmBatch *&value, int indicator) {   // :46-57
        std::unique_lock<std::mutex> lk(m_);
        avail_cv_.wait(lk, [this, indicator] { return full_ && !taken_[indicator]; });
        value = slot_;
        taken_[indicator] = true;
        if (taken_[0] && taken_[1]) full_ = false;
    }

    void prepare(int indicator) {   // :65-74
        std::lock_guard<std::mutex> lk(m_);
        if (indicator == 0 || indicator == 1) released_[indicator] = true;
        if (released_[0] && released_[1] && slot_) {   // both done: the slot's batch is free again
            free_.push_back(slot_);
            slot_ = nullptr;
        }
        free_cv_.notify_all();
    }

private:
    FmBatch *slot_ = nullptr;
    std::vector<FmBatch *> free_;
    bool released_[2] = {true, true};
    bool taken_[2] = {false, false};
    bool full_ = false;
    std::mutex m_;
    std::condition_variable avail_cv_, free_cv_;
};

#endif
