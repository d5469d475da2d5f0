// am_par.h -- host worker threads for the per-document host stages of the batched calls (the sync
// protocol's graph queries and message building, the graph indexing): f(i) for i in [0, n) on
// AM_HOST_THREADS threads (default: the machine's, at most 16), in chunks of 64 items.
#pragma once
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

inline unsigned am_host_threads() {
  const char* e = getenv("AM_HOST_THREADS");
  unsigned n = e ? (unsigned)atoi(e) : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  return n ? n : 1;
}

template <class F>
void am_par_for(size_t n, F f) {
  const unsigned nt = am_host_threads();
  if (nt <= 1 || n < 128) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  // an exception on a worker (std::bad_alloc, ...) stops the loop and is rethrown on the calling
  // thread after the join, as the serial loop would throw it, instead of std::terminate
  std::atomic<size_t> next{0};
  std::atomic<bool> stop{false};
  std::exception_ptr first;
  std::mutex mu;
  auto work = [&]() {
    for (;;) {
      const size_t i0 = next.fetch_add(64);
      if (i0 >= n || stop.load(std::memory_order_relaxed)) return;
      try {
        for (size_t i = i0; i < std::min(n, i0 + 64); i++) f(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(mu);
        if (!first) first = std::current_exception();
        stop = true;
        return;
      }
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  if (first) std::rethrow_exception(first);
}

// Deferred reclamation: the per-document buffers a batched call leaves (millions of small vectors
// for 200k handles: 140-400 ms of frees on the workers, measured) are destroyed on one background
// thread instead of on the caller's critical path. AM_RECLAIM=0 destroys them in place, on the
// workers, as before. The thread is started on first use (never before a fork of the caller's).
class AmReclaimer {
 public:
  // at most kMaxQueued batches wait for the thread: a caller that outruns it frees in its own
  // time (backpressure) instead of letting the queued memory grow without bound
  static constexpr size_t kMaxQueued = 8;
  static AmReclaimer& get() {
    static std::atomic<AmReclaimer*> cur{nullptr};
    AmReclaimer* r = cur.load();
    // a forked child inherits the object but not its thread: it starts a reclaimer of its own (the
    // parent's is leaked in the child; its mutex may have been held at the fork)
    if (!r || r->pid_ != getpid()) {
      static std::mutex mk;
      std::lock_guard<std::mutex> g(mk);
      r = cur.load();
      if (!r || r->pid_ != getpid()) {
        r = new AmReclaimer();  // never destroyed: the thread may outlive main()
        cur.store(r);
      }
    }
    return *r;
  }
  void push(std::function<void()> f) {
    {
      std::unique_lock<std::mutex> g(m_);
      if (q_.size() >= kMaxQueued) {
        g.unlock();
        f();  // the queue is full: free inline
        return;
      }
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  AmReclaimer() : pid_(getpid()) { std::thread([this] { run(); }).detach(); }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  const pid_t pid_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};
// hands the vector's elements to the reclaimer (v is left empty)
template <class T>
void am_reclaim(std::vector<T>& v) {
  static const bool on = [] { const char* e = getenv("AM_RECLAIM"); return !(e && e[0] == '0'); }();
  if (!on) {
    am_par_for(v.size(), [&](size_t i) { v[i] = T(); });
    std::vector<T>().swap(v);
    return;
  }
  auto p = std::make_shared<std::vector<T>>(std::move(v));
  v.clear();
  AmReclaimer::get().push([p]() mutable { p.reset(); });
}
