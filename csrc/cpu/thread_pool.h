// Persistent worker pool for the CPU backend. Unlike the reference executor, which creates and
// joins nThreads-1 pthreads on every forward (nn-executor.cpp:178-186), the workers live for the
// lifetime of the backend and are woken per parallel region.
#pragma once

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dl {

class ThreadPool {
  public:
    explicit ThreadPool(int nThreads);
    ~ThreadPool();
    int size() const { return n_; }
    // fn(threadIndex, nThreads) on every thread, caller participates as thread 0.
    void run(const std::function<void(int, int)> &fn);
    // Splits [0, count) into contiguous ranges, one per thread.
    void parallelFor(long count, const std::function<void(long, long)> &fn);

  private:
    void worker(int idx);
    int n_;
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_, doneCv_;
    const std::function<void(int, int)> *job_ = nullptr;
    long generation_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

}  // namespace dl
