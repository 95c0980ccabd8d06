// threadsafequeue.h (drop-in) -- the reference's one-slot broadcast mailbox between the RF
// front-end producer and the two consumers (audio = indicator 0, RDS = indicator 1), with the same
// protocol (reference include/threadsafequeue.h:8-76):
//   push(v)            waits until both consumers have called prepare() for the previous payload,
//                      deletes that payload, publishes v to both consumers
//   wait_and_pop(v,i)  waits for a payload consumer i has not read yet
//   prepare(i)         consumer i is done with the payload (the producer may replace it)
#ifndef SDR_DROPIN_THREADSAFEQUEUE_H
#define SDR_DROPIN_THREADSAFEQUEUE_H

#include <condition_variable>
#include <mutex>

template <typename T>
class ThreadSafeQueue {
public:
    ThreadSafeQueue() = default;
    ThreadSafeQueue(const ThreadSafeQueue &) = delete;
    ThreadSafeQueue &operator=(const ThreadSafeQueue &) = delete;

    void push(const T value) {
        std::unique_lock<std::mutex> lk(m_);
        free_cv_.wait(lk, [this] { return released_[0] && released_[1]; });
        if (slot_) delete slot_;
        slot_ = value;
        released_[0] = released_[1] = false;
        taken_[0] = taken_[1] = false;
        full_ = true;
        avail_cv_.notify_all();
    }

    void wait_and_pop(T &value, int indicator) {
        std::unique_lock<std::mutex> lk(m_);
        avail_cv_.wait(lk, [this, indicator] { return full_ && !taken_[indicator]; });
        value = slot_;
        taken_[indicator] = true;
        if (taken_[0] && taken_[1]) full_ = false;
    }

    void prepare(int indicator) {
        std::lock_guard<std::mutex> lk(m_);
        if (indicator == 0 || indicator == 1) released_[indicator] = true;
        free_cv_.notify_all();
    }

private:
    T slot_ = nullptr;
    bool released_[2] = {true, true};
    bool taken_[2] = {false, false};
    bool full_ = false;
    std::mutex m_;
    std::condition_variable avail_cv_, free_cv_;
};

#endif
