// A fixed pool of host worker threads for the per-image entropy coding (rANS encode after the
// network, rANS decode between the 20 slice phases).  Every lane submits its images' jobs here
// instead of spawning threads per phase; run() blocks until the caller's batch is done and
// rethrows the first exception of that batch.  Jobs are tagged encode / decode and, by default, the
// encodes are served first: a lane's decompress cannot start before its images' streams exist, while
// a queued per-phase decode only delays one lane's next small kernels (measured, 4 request streams x
// 2 lanes, three alternating pairs: 89.5 img/s encodes-first against 88.4 FIFO; decodes-first 86.9
// against FIFO 87.8).  $MLIC_POOL_PRIO: 2 (default) encodes first, 1 decodes first, 0 one FIFO.
#pragma once
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mlic {

class HostPool {
 public:
  explicit HostPool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  // runs fn(0..n-1) on the pool (the caller runs one share itself) and waits
  enum Kind { ENCODE = 0, DECODE = 1 };
  void run(int n, const std::function<void(int)>& fn, Kind kind = ENCODE) {
    if (n <= 1) {
      if (n == 1) fn(0);
      return;
    }
    struct Batch {
      std::mutex m;
      std::condition_variable cv;
      int left;
      std::exception_ptr err;
    } batch;
    batch.left = n - 1;
    {
      std::lock_guard<std::mutex> g(m_);
      const int pr = prio();
      const bool urgent = (pr == 1 && kind == DECODE) || (pr == 2 && kind == ENCODE);
      auto& q = urgent ? uq_ : q_;
      for (int i = 1; i < n; ++i)
        q.push_back([&batch, &fn, i] {
          std::exception_ptr e;
          try {
            fn(i);
          } catch (...) {
            e = std::current_exception();
          }
          std::lock_guard<std::mutex> g2(batch.m);
          if (e && !batch.err) batch.err = e;
          if (--batch.left == 0) batch.cv.notify_all();
        });
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      fn(0);
    } catch (...) {
      mine = std::current_exception();
    }
    std::unique_lock<std::mutex> g(batch.m);
    batch.cv.wait(g, [&] { return batch.left == 0; });
    if (mine) std::rethrow_exception(mine);
    if (batch.err) std::rethrow_exception(batch.err);
  }

 private:
  static int prio() {
    static const int p = [] {
      const char* e = std::getenv("MLIC_POOL_PRIO");
      return e ? std::atoi(e) : 2;
    }();
    return p;
  }
  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return stop_ || !q_.empty() || !uq_.empty(); });
        if (stop_ && q_.empty() && uq_.empty()) return;
        auto& q = uq_.empty() ? q_ : uq_;
        job = std::move(q.front());
        q.pop_front();
      }
      job();
    }
  }
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_, uq_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

}  // namespace mlic
