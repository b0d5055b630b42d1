#include "thread_pool.h"

namespace dl {

ThreadPool::ThreadPool(int nThreads) : n_(nThreads < 1 ? 1 : nThreads) {
    for (int i = 1; i < n_; i++) threads_.emplace_back([this, i] { worker(i); });
}

ThreadPool::~ThreadPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_) t.join();
}

void ThreadPool::worker(int idx) {
    long seen = 0;
    while (true) {
        const std::function<void(int, int)> *job;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
            if (stop_) return;
            seen = generation_;
            job = job_;
        }
        (*job)(idx, n_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) doneCv_.notify_one();
        }
    }
}

void ThreadPool::run(const std::function<void(int, int)> &fn) {
    if (n_ == 1) {
        fn(0, 1);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = &fn;
        pending_ = n_ - 1;
        generation_++;
    }
    cv_.notify_all();
    fn(0, n_);
    std::unique_lock<std::mutex> lk(mu_);
    doneCv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
}

void ThreadPool::parallelFor(long count, const std::function<void(long, long)> &fn) {
    if (count <= 0) return;
    run([&](int t, int nt) {
        const long slice = count / nt, rest = count % nt;
        const long s = t * slice + (t < rest ? t : rest);
        const long e = s + slice + (t < rest ? 1 : 0);
        if (s < e) fn(s, e);
    });
}

}  // namespace dl
