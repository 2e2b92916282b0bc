// ref_htree.h — QueueModelHistoryTree::computeQueueDelay restated on the
// reference's own IntervalTree and QueueModelMG1 (queue_model_history_tree.cc
// needs Boost through config.hpp).  Shared by ref_harness.cc and
// coh_harness.cc.  TEST INFRASTRUCTURE ONLY.
#pragma once
#include <vector>
#include <utility>
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

  RefHistoryTree(UInt64 mp, SInt32 ms, bool an) : min_proc(mp), max_size(ms), analytical(an), analytical_requests(0) {
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
    return qd;
  }
};

