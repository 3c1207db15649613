// kflow.h — the slice of bwa-flow's kestrelFlow runtime that the SW stage
// plugs into, restated on std::thread (the reference's is boost-based:
// kflow/include/kflow/{Queue,Stage,MapStage,MapPartitionStage,Pipeline}.h).
//
// Same names and the same contract, so ChainsToRegionsGPU compiles against
// either this file or the reference's kflow unchanged:
//   Queue<U,DEPTH>          bounded MPMC queue: push/pop block, async_* poll
//   Stage<U,V,IN,OUT>       typed queues of a stage
//   MapStage<U,V>           dynamic CPU workers, V compute(U const&); when an
//                           accelerator back end is attached and useAccx(),
//                           inputs are handed to its load queue while that
//                           queue is short (MapStage.h:103-111); when the
//                           accelerator is switched off the load queue is
//                           drained back into the CPU workers (MapStage.h:84-92)
//   MapPartitionStage<U,V>  static workers running compute(wid) with
//                           getInput()/pushOutput() (MapPartitionStage.h)
//   Pipeline                addStage / addAccxBckStage / start / wait
//                           (Pipeline.h:36,150-180)
// Not restated: MegaPipe, MPI channels, occupancy-based thread scheduling.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

namespace kestrelFlow {

class QueueBase {
 public:
  virtual ~QueueBase() = default;
  virtual bool empty() = 0;
  virtual int get_size() = 0;
};

template <typename U, int DEPTH = 64>
class Queue : public QueueBase {
 public:
  explicit Queue(int depth = DEPTH) : cap_(depth > 0 ? depth : 1) {}
  bool empty() override { return get_size() == 0; }
  int get_size() override {
    std::lock_guard<std::mutex> g(m_);
    return (int)q_.size();
  }
  int get_capacity() const { return cap_; }
  bool almost_full() { return get_size() >= cap_ / 2; }
  void push(U item) {
    std::unique_lock<std::mutex> g(m_);
    not_full_.wait(g, [&] { return (int)q_.size() < cap_; });
    q_.push_back(std::move(item));
    not_empty_.notify_one();
  }
  void pop(U& item) {
    std::unique_lock<std::mutex> g(m_);
    not_empty_.wait(g, [&] { return !q_.empty(); });
    take(item);
  }
  bool async_push(U item) {
    std::lock_guard<std::mutex> g(m_);
    if ((int)q_.size() >= cap_) return false;
    q_.push_back(std::move(item));
    not_empty_.notify_one();
    return true;
  }
  bool async_pop(U& item) {
    std::lock_guard<std::mutex> g(m_);
    if (q_.empty()) return false;
    take(item);
    return true;
  }

 private:
  void take(U& item) {
    item = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
  }
  const int cap_;
  std::mutex m_;
  std::condition_variable not_empty_, not_full_;
  std::deque<U> q_;
};

class Pipeline;

class StageBase {
  friend class Pipeline;

 public:
  StageBase(int num_workers = 1, bool is_dyn = true) : num_workers_(num_workers), is_dynamic_(is_dyn) {}
  virtual ~StageBase() = default;

  int getMaxNumThreads() const { return num_workers_; }
  int getNumActiveThreads() const { return active_.load(); }
  bool isDynamic() const { return is_dynamic_; }
  bool useAccx() const { return use_accx_.load(); }
  void setUseAccx(bool f) { use_accx_.store(f); }
  StageBase* getAccxStage() { return accx_backend_stage_; }
  // every worker has returned from its loop
  bool workersDone() const { return started_.load() && active_.load() == 0; }

  StageBase* accx_backend_stage_ = nullptr;
  float accx_priority_ = 1.0f;

  void start() {
    started_.store(true);
    active_.store(num_workers_);
    for (int i = 0; i < num_workers_; ++i)
      threads_.emplace_back([this, i] {
        worker_func(i);
        active_.fetch_sub(1);
      });
  }
  void wait() {
    for (auto& t : threads_) t.join();
    threads_.clear();
  }

 protected:
  // no more input will ever arrive (all upstream producers are done)
  bool isFinal() const { return final_pred_ ? final_pred_() : true; }
  virtual bool inputQueueEmpty() = 0;
  virtual void worker_func(int wid) = 0;
  // kflow's StageBase::finalize() (called once per worker on exit): upstream
  // completion is tracked by final_pred_ here, so there is nothing to signal
  void finalize() {}

  std::function<bool()> final_pred_;
  std::shared_ptr<QueueBase> input_queue_, output_queue_, accx_load_queue_;

 private:
  int num_workers_;
  bool is_dynamic_;
  std::atomic<bool> use_accx_{false}, started_{false};
  std::atomic<int> active_{0};
  std::vector<std::thread> threads_;
};

template <typename U, typename V, int IN_DEPTH = 64, int OUT_DEPTH = 64>
class Stage : public StageBase {
  friend class Pipeline;

 public:
  using In = U;
  using Out = V;
  static constexpr int InDepth = IN_DEPTH, OutDepth = OUT_DEPTH;
  Stage(int n = 1, bool is_dyn = true) : StageBase(n, is_dyn) {}
  Queue<U, IN_DEPTH>* getInputQueue() { return cast<U, IN_DEPTH>(input_queue_); }
  Queue<V, OUT_DEPTH>* getOutputQueue() { return cast<V, OUT_DEPTH>(output_queue_); }
  Queue<U, IN_DEPTH>* getAccxQueue() { return cast<U, IN_DEPTH>(accx_load_queue_); }

 protected:
  bool inputQueueEmpty() override { return !input_queue_ || input_queue_->empty(); }

 private:
  template <typename T, int D>
  static Queue<T, D>* cast(const std::shared_ptr<QueueBase>& q) {
    if (!q) return nullptr;
    auto* p = dynamic_cast<Queue<T, D>*>(q.get());
    if (!p) throw std::logic_error("kflow: queue type mismatch");
    return p;
  }
};

// the reference's MapStage idles 100 us between polls of its input queue
// (kflow/include/kflow/MapStage.h:186-189)
inline void idle_wait() { std::this_thread::sleep_for(std::chrono::microseconds(100)); }

// CPU stage with an optional accelerator back end (ChainsToRegions is one)
template <typename U, typename V, int IN_DEPTH = 64, int OUT_DEPTH = 64>
class MapStage : public Stage<U, V, IN_DEPTH, OUT_DEPTH> {
 public:
  MapStage(int n = 1, bool is_dyn = true) : Stage<U, V, IN_DEPTH, OUT_DEPTH>(n, is_dyn) {}
  virtual V compute(U const& input) = 0;

 protected:
  void worker_func(int) override {
    auto* in = this->getInputQueue();
    auto* out = this->getOutputQueue();
    StageBase* accx = this->accx_backend_stage_;
    for (;;) {
      U item;
      if (accx && (!this->useAccx() || accx->workersDone())) {  // accelerator gone: take its backlog back
        auto* aq = this->getAccxQueue();
        while (aq->async_pop(item)) in->push(std::move(item));
      }
      if (!in->async_pop(item)) {
        // exit only once nothing can come back from the accelerator either
        if (this->isFinal() && in->empty() && (!accx || accx->workersDone()) &&
            (!accx || this->getAccxQueue()->empty()))
          break;
        idle_wait();
        continue;
      }
      if (accx && this->useAccx() && !accx->workersDone()) {
        auto* aq = this->getAccxQueue();
        const int sz = aq->get_size();
        if (sz < aq->get_capacity() && sz <= accx->getNumActiveThreads() * this->accx_priority_ &&
            aq->async_push(item))
          continue;
      }
      V r = compute(item);
      if (out) out->push(std::move(r));
    }
    this->finalize();
  }
};

// static-worker stage driven by compute(wid) (the FPGA/GPU back ends)
template <typename U, typename V, int IN_DEPTH = 64, int OUT_DEPTH = 64>
class MapPartitionStage : public Stage<U, V, IN_DEPTH, OUT_DEPTH> {
 public:
  MapPartitionStage(int n = 1, bool is_dyn = true) : Stage<U, V, IN_DEPTH, OUT_DEPTH>(n, is_dyn) {}

 protected:
  virtual void compute(int wid) = 0;
  bool getInput(U& item) {
    auto* q = this->getInputQueue();
    return q && q->async_pop(item);
  }
  void pushOutput(V const& item) {
    if (auto* q = this->getOutputQueue()) q->push(item);
  }
  void worker_func(int wid) override {
    compute(wid);
    this->finalize();
  }
};

// A linear pipeline of stages; the caller feeds stage 0 through input() and
// calls closeInput() after the last record, and drains the last stage's
// output() (or leaves it unbounded-consumed by a following stage).
class Pipeline {
 public:
  explicit Pipeline(int n_stages) : stages_(n_stages, nullptr), accx_(n_stages, nullptr) {}

  template <typename S>
  bool addStage(int idx, S* stage) {
    if (idx < 0 || idx >= (int)stages_.size() || stages_[idx]) return false;
    static_assert(S::InDepth == 64 && S::OutDepth == 64, "kflow: stages use COMPUTE_DEPTH (64) queues");
    stages_[idx] = stage;
    using U = typename S::In;
    using V = typename S::Out;
    if (idx == 0) stage->input_queue_ = std::make_shared<Queue<U, 64>>(64);
    else stage->input_queue_ = stages_[idx - 1]->output_queue_;
    stage->output_queue_ = std::make_shared<Queue<V, 64>>(64);
    return true;
  }

  // accelerator back end of stage idx: a private load queue fed by the CPU
  // stage, the CPU stage's output queue (Pipeline.h:150-180)
  template <typename S>
  bool addAccxBckStage(int idx, S* accx, float init_priority = 1.0f) {
    StageBase* cpu = stages_.at(idx);
    if (!cpu || accx_[idx]) return false;
    static_assert(S::InDepth == 64, "kflow: stages use COMPUTE_DEPTH (64) queues");
    using U = typename S::In;
    const int depth = std::max(1, (int)((init_priority + 1) * accx->getMaxNumThreads()));
    accx->input_queue_ = std::make_shared<Queue<U, 64>>(depth);
    accx->output_queue_ = cpu->output_queue_;
    cpu->accx_load_queue_ = accx->input_queue_;
    cpu->accx_backend_stage_ = accx;
    cpu->accx_priority_ = init_priority;
    cpu->setUseAccx(true);
    accx_[idx] = accx;
    return true;
  }

  template <typename U>
  Queue<U, 64>* input() { return dynamic_cast<Queue<U, 64>*>(stages_.at(0)->input_queue_.get()); }
  template <typename V>
  Queue<V, 64>* output() { return dynamic_cast<Queue<V, 64>*>(stages_.back()->output_queue_.get()); }
  void closeInput() { input_closed_.store(true); }

  void start() {
    for (size_t i = 0; i < stages_.size(); ++i) {
      StageBase* s = stages_[i];
      if (!s) throw std::logic_error("kflow: pipeline has an empty stage slot");
      if (i == 0) {
        s->final_pred_ = [this] { return input_closed_.load(); };
      } else {
        StageBase* up = stages_[i - 1];
        StageBase* ua = accx_[i - 1];
        s->final_pred_ = [up, ua] { return up->workersDone() && (!ua || ua->workersDone()); };
      }
      if (StageBase* a = accx_[i]) {  // no more inputs once the CPU stage's own input is exhausted
        a->final_pred_ = [s] { return s->isFinal() && s->inputQueueEmpty(); };
      }
    }
    for (size_t i = 0; i < stages_.size(); ++i) {
      stages_[i]->start();
      if (accx_[i]) accx_[i]->start();
    }
  }
  void wait() {
    for (size_t i = 0; i < stages_.size(); ++i) {
      if (accx_[i]) accx_[i]->wait();
      stages_[i]->wait();
    }
  }

 private:
  std::vector<StageBase*> stages_, accx_;
  std::atomic<bool> input_closed_{false};
};

}  // namespace kestrelFlow
