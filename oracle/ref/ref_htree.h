// ref_htree.h — QueueModelHistoryTree::computeQueueDelay restated on the
// reference's own IntervalTree and QueueModelMG1 (queue_model_history_tree.cc
// needs Boost through config.hpp).  Shared by ref_harness.cc and
// coh_harness.cc.  TEST INFRASTRUCTURE ONLY.
#pragma once
#include <vector>
#include <utility>
#include <algorithm>
#include "interval_tree.h"
#include "queue_model_m_g_1.h"

#ifndef CHECK
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "ref harness: check failed %s:%d: %s\n", __FILE__, __LINE__, #c); exit(2); } } while (0)
#endif

// QueueModelHistoryTree::computeQueueDelay (queue_model_history_tree.cc:44-126)
// on the reference IntervalTree / QueueModelMG1
// --------------------------------------------------------------------------
struct RefHistoryTree {
  UInt64 min_proc; SInt32 max_size; bool analytical;
  IntervalTree::Node* blocks; vector<SInt32> free_list; SInt32 tail;
  IntervalTree* tree; QueueModelMG1 mg1; UInt64 analytical_requests;
  UInt64 util, last_req;                      // QueueModel utilization counters (queue_model.cc:41-55)

  RefHistoryTree(UInt64 mp, SInt32 ms, bool an)
      : min_proc(mp), max_size(ms), analytical(an), analytical_requests(0), util(0), last_req(0) {
    blocks = new IntervalTree::Node[ms];                          // allocateMemory (:129-137)
    free_list.resize(ms); for (SInt32 i = 0; i < ms; ++i) free_list[i] = i;
    tail = ms - 1;
    tree = new IntervalTree(alloc(0, UINT64_MAX));
  }
  ~RefHistoryTree() { delete tree; delete[] blocks; }
  IntervalTree::Node* alloc(UInt64 a, UInt64 b) {                // allocateNode (:146-157)
    CHECK(tail >= 0);
    IntervalTree::Node* n = &blocks[free_list[tail--]];
    n->initialize(make_pair(a, b));
    return n;
  }
  void release(IntervalTree::Node* n) { free_list[++tail] = (SInt32)(n - blocks); CHECK(tail < max_size); }

  UInt64 delay(UInt64 t, UInt64 p) {
    UInt64 qd = UINT64_MAX;
    IntervalTree::Node* mn = tree->search(make_pair((UInt64)0, (UInt64)1));
    if (tree->size() >= (UInt32)max_size) release(tree->remove(mn));
    mn = tree->search(make_pair((UInt64)0, (UInt64)1));
    if (analytical && (mn->interval.first > (t + p))) {
      analytical_requests++;
      qd = mg1.computeQueueDelay(t, p);
    } else {
      IntervalTree::Node* n = tree->search(make_pair(t, t + p));
      CHECK(n);
      CHECK((t + p) <= n->interval.second);
      if (t >= n->interval.first) {
        qd = 0;
        if ((t - n->interval.first) >= min_proc) {
          if ((n->interval.second - (t + p)) >= min_proc) tree->insert(alloc(t + p, n->interval.second));
          n->interval.second = t;
        } else {
          if ((n->interval.second - (t + p)) >= min_proc) { n->interval.first = t + p; n->key = n->interval.first; }
          else release(tree->remove(n));
        }
      } else {
        qd = n->interval.first - t;
        if ((n->interval.second - (n->interval.first + p)) >= min_proc) {
          n->interval.first = n->interval.first + p; n->key = n->interval.first;
        } else release(tree->remove(n));
      }
    }
    CHECK(qd != UINT64_MAX);
    mg1.updateQueue(t, p, qd);
    util += p;                                  // updateQueueUtilizationCounters (queue_model.cc:49-55)
    last_req = std::max<UInt64>(last_req, t + qd + p);
    return qd;
  }
};


// --------------------------------------------------------------------------
// QueueModelHistoryList::computeQueueDelay (queue_model_history_list.cc:40-134)
// on std::list — the container the reference uses, with its iterator
// semantics (erase returns the next node, insert goes before it, -- on
// begin() wraps to the sentinel) — and the reference QueueModelMG1.  The
// reference file reads its parameters through Sim()->getCfg() (Boost), so
// the glue is restated here.
// --------------------------------------------------------------------------
#include <list>
struct RefHistoryList {
  typedef std::list<std::pair<UInt64, UInt64> > L;
  UInt64 min_proc; UInt32 max_size; bool analytical, interleaving;
  L fl; QueueModelMG1 mg1; UInt64 analytical_requests;

  RefHistoryList(UInt64 mp, UInt32 ms, bool an, bool il)
      : min_proc(mp), max_size(ms), analytical(an), interleaving(il), analytical_requests(0) {
    fl.push_back(std::make_pair((UInt64)0, (UInt64)UINT64_MAX));
  }
  UInt64 scan(UInt64 t, UInt64 p) {
    CHECK(fl.size() <= max_size);
    UInt64 qd = 0;
    for (L::iterator it = fl.begin(); it != fl.end(); ++it) {
      const UInt64 a = it->first, b = it->second;
      if (t >= a && t + p <= b) {
        it = fl.erase(it);
        if (t - a >= min_proc) fl.insert(it, std::make_pair(a, t));
        if (b - (t + p) >= min_proc) fl.insert(it, std::make_pair(t + p, b));
        break;
      }
      if (t < a && a + p <= b) {
        qd += a - t;
        it = fl.erase(it);
        if (b - (a + p) >= min_proc) fl.insert(it, std::make_pair(a + p, b));
        break;
      }
      if (!interleaving) continue;
      if (t >= a && t < b) {
        it = fl.erase(it);
        if (t - a >= min_proc) fl.insert(it, std::make_pair(a, t));
        --it;
        t = b;
        p -= (b - t);          // as the reference: after t moved, this subtracts 0
      } else if (t < a) {
        it = fl.erase(it);
        --it;
        qd += a - t;
        t = b;
        p -= (b - a);
      }
    }
    if (fl.size() > max_size) fl.erase(fl.begin());
    return qd;
  }
  UInt64 delay(UInt64 t, UInt64 p) {
    CHECK(fl.size() >= 1);
    UInt64 qd;
    if (analytical && (t + p) < fl.front().first) { analytical_requests++; qd = mg1.computeQueueDelay(t, p); }
    else qd = scan(t, p);
    mg1.updateQueue(t, p, qd);
    return qd;
  }
};

// --------------------------------------------------------------------------
// QueueModelBasic::computeQueueDelay (queue_model_basic.cc:34-61) on the
// reference's own MovingAverage<UInt64> (common/misc/moving_average.h +
// modulo_num.cc); avg = "arithmetic_mean" / "median" / "" (disabled).
// --------------------------------------------------------------------------
#include "moving_average.h"
struct RefBasic {
  UInt64 queue_time; MovingAverage<UInt64>* ma;
  RefBasic(const char* avg, UInt32 window) : queue_time(0), ma(NULL) {
    if (avg[0]) { ma = MovingAverage<UInt64>::createAvgType(avg, window); CHECK(ma); }
  }
  ~RefBasic() { delete ma; }
  UInt64 delay(UInt64 t, UInt64 p) {
    const UInt64 ref = ma ? ma->compute(t) : t;
    const UInt64 qd = queue_time > ref ? queue_time - ref : 0;
    queue_time = std::max(queue_time, ref) + p;
    return qd;
  }
};
