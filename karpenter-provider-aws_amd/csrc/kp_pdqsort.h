// kp_pdqsort.h — Go 1.24 sort.Slice (src/sort/zsortfunc.go pdqsort_func) restated for one device lane.
//
// Upstream Scheduler.add sorts s.newNodeClaims with sort.Slice by len(Pods) before every
// addToInflightNode. sort.Slice is NOT stable; the permutation of equal keys is what pdqsort does, so
// the device replays the exact algorithm (insertion sort <= 12, ninther pivot, partial insertion sort,
// partitionEqual, breakPatterns xorshift(len), heapsort fallback). Recursion is replaced by an explicit
// stack (depth <= 2*log2(n)+2).
#pragma once

template <class LS>
struct DevPDQ {
  const LS& d;
  __device__ void insertionSort(int a, int b) const {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
  }
  __device__ void siftDown(int lo, int hi, int first) const {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
      if (!d.Less(first + root, first + child)) return;
      d.Swap(first + root, first + child);
      root = child;
    }
  }
  __device__ void heapSort(int a, int b) const {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      d.Swap(first, first + i);
      siftDown(lo, i, first);
    }
  }
  __device__ static int bitsLen(unsigned long long x) { return x == 0 ? 0 : 64 - __builtin_clzll(x); }
  __device__ void breakPatterns(int a, int b) const {
    int length = b - a;
    if (length >= 8) {
      unsigned long long random = (unsigned long long)length;
      unsigned long long modulus = 1ull << bitsLen((unsigned long long)length);
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        random ^= random << 13;
        random ^= random >> 7;
        random ^= random << 17;
        int other = (int)((unsigned)random & (unsigned)(modulus - 1));
        if (other >= length) other -= length;
        d.Swap(idx - 1 + i, a + other);
      }
    }
  }
  __device__ void order2(int& a, int& b, int* swaps) const {
    if (d.Less(b, a)) {
      (*swaps)++;
      int t = a;
      a = b;
      b = t;
    }
  }
  __device__ int median(int a, int b, int c, int* swaps) const {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  __device__ int choosePivot(int a, int b, int* hint) const {
    int l = b - a, swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) {
        i = median(i - 1, i, i + 1, &swaps);
        j = median(j - 1, j, j + 1, &swaps);
        k = median(k - 1, k, k + 1, &swaps);
      }
      j = median(i, j, k, &swaps);
    }
    *hint = swaps == 0 ? 0 : (swaps == 12 ? 1 : 2);  // increasing / decreasing / unknown
    return j;
  }
  __device__ void reverseRange(int a, int b) const {
    int i = a, j = b - 1;
    while (i < j) d.Swap(i++, j--);
  }
  __device__ bool partialInsertionSort(int a, int b) const {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      while (i < b && !d.Less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < 50) return false;
      d.Swap(i, i - 1);
      if (i - a >= 2) {
        for (int k = i - 1; k >= 1; k--) {
          if (!d.Less(k, k - 1)) break;
          d.Swap(k, k - 1);
        }
      }
      if (b - i >= 2) {
        for (int k = i + 1; k < b; k++) {
          if (!d.Less(k, k - 1)) break;
          d.Swap(k, k - 1);
        }
      }
    }
    return false;
  }
  __device__ int partitionEqual(int a, int b, int pivot) const {
    d.Swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !d.Less(a, i)) i++;
      while (i <= j && d.Less(a, j)) j--;
      if (i > j) break;
      d.Swap(i, j);
      i++;
      j--;
    }
    return i;
  }
  __device__ int partition(int a, int b, int pivot, bool* already) const {
    d.Swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    if (i > j) {
      d.Swap(j, a);
      *already = true;
      return j;
    }
    d.Swap(i, j);
    i++;
    j--;
    for (;;) {
      while (i <= j && d.Less(i, a)) i++;
      while (i <= j && !d.Less(j, a)) j--;
      if (i > j) break;
      d.Swap(i, j);
      i++;
      j--;
    }
    d.Swap(j, a);
    *already = false;
    return j;
  }
  // pdqsort_func with the recursive call on the smaller side turned into an explicit stack frame.
  __device__ void run(int a0, int b0, int limit0) const {
    struct Frame {
      int a, b, limit;
      bool wasBalanced, wasPartitioned;
      int resume_a, resume_b;  // the caller's loop state to restore after the child returns
      bool child_left;
    };
    Frame st[40];
    int sp = 0;
    int a = a0, b = b0, limit = limit0;
    bool wasBalanced = true, wasPartitioned = true;
    for (;;) {
      // loop body of pdqsort_func
      int length = b - a;
      bool done = false;
      if (length <= 12) {
        insertionSort(a, b);
        done = true;
      } else if (limit == 0) {
        heapSort(a, b);
        done = true;
      } else {
        if (!wasBalanced) {
          breakPatterns(a, b);
          limit--;
        }
        int hint;
        int pivot = choosePivot(a, b, &hint);
        if (hint == 1) {
          reverseRange(a, b);
          pivot = (b - 1) - (pivot - a);
          hint = 0;
        }
        if (wasBalanced && wasPartitioned && hint == 0) {
          if (partialInsertionSort(a, b)) done = true;
        }
        if (!done) {
          if (a > 0 && !d.Less(a - 1, pivot)) {
            a = partitionEqual(a, b, pivot);
            continue;  // same frame, loop again
          }
          bool already = false;
          int mid = partition(a, b, pivot, &already);
          wasPartitioned = already;
          int leftLen = mid - a, rightLen = b - mid;
          int balanceThreshold = length / 8;
          Frame f;
          f.limit = limit;
          f.wasPartitioned = wasPartitioned;
          if (leftLen < rightLen) {
            f.wasBalanced = leftLen >= balanceThreshold;
            f.resume_a = mid + 1;
            f.resume_b = b;
            f.child_left = true;
            st[sp++] = f;
            // recurse on [a, mid) with fresh flags
            b = mid;
          } else {
            f.wasBalanced = rightLen >= balanceThreshold;
            f.resume_a = a;
            f.resume_b = mid;
            f.child_left = false;
            st[sp++] = f;
            a = mid + 1;
          }
          wasBalanced = true;
          wasPartitioned = true;
          continue;
        }
      }
      // this frame finished: pop the parent and continue its loop
      if (sp == 0) return;
      Frame f = st[--sp];
      a = f.resume_a;
      b = f.resume_b;
      limit = f.limit;
      wasBalanced = f.wasBalanced;
      wasPartitioned = f.wasPartitioned;
    }
  }
};

template <class LS>
__device__ void go_sort_slice(const LS& ls, int n) {
  DevPDQ<LS> p{ls};
  p.run(0, n, DevPDQ<LS>::bitsLen((unsigned long long)n));
}
