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

// Persistent host workers for am_par_for: a call hands its loop to threads that already exist
// (spawning and joining 15 threads cost a millisecond or more per call, and the batched calls make
// several). One loop at a time owns the workers; a loop that finds them busy, or that runs on a
// worker itself (nested), starts threads of its own as before. A forked child gets a pool of its own.
class AmPool {
 public:
  static AmPool& get() {
    static std::atomic<AmPool*> cur{nullptr};
    AmPool* p = cur.load();
    if (!p || p->pid_ != getpid()) {
      static std::mutex mk;
      std::lock_guard<std::mutex> g(mk);
      p = cur.load();
      if (!p || p->pid_ != getpid()) {
        p = new AmPool(am_host_threads());  // never destroyed: its threads may outlive main()
        cur.store(p);
      }
    }
    return *p;
  }
  static bool on_worker() { return worker_flag(); }
  // runs work() on the calling thread and every worker; false when the workers are busy
  bool run(const std::function<void()>& work) {
    std::unique_lock<std::mutex> own(owner_, std::try_to_lock);
    if (!own.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(m_);
      work_ = &work;
      active_ = (unsigned)th_.size();
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return active_ == 0; });
    work_ = nullptr;
    return true;
  }

 private:
  explicit AmPool(unsigned nt) : pid_(getpid()) {
    for (unsigned t = 1; t < nt; t++) th_.emplace_back([this] { loop(); });
    for (auto& t : th_) t.detach();
  }
  static bool& worker_flag() {
    static thread_local bool f = false;
    return f;
  }
  void loop() {
    worker_flag() = true;
    uint64_t seen = 0;
    for (;;) {
      const std::function<void()>* w;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        w = work_;
      }
      (*w)();
      std::lock_guard<std::mutex> g(m_);
      if (--active_ == 0) done_.notify_one();
    }
  }
  const pid_t pid_;
  std::vector<std::thread> th_;
  std::mutex owner_, m_;
  std::condition_variable cv_, done_;
  const std::function<void()>* work_ = nullptr;
  unsigned active_ = 0;
  uint64_t gen_ = 0;
};

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
  const std::function<void()> work = [&]() {
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
  if (AmPool::on_worker() || !AmPool::get().run(work)) {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
  }
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
