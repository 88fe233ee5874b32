// Grow-only scratch arena with allocation generations (host-only bookkeeping,
// no HIP types: tests/cpp/arena_check.cpp builds it with a malloc backend).
//
// Why generations: a cache keyed by a device ADDRESS is wrong once the buffer
// behind it is freed and hipMalloc hands the same address to another buffer
// (scratch regrowth does exactly that).  An inverse NTT once ran on a stale
// forward twiddle pyramid after a 17 -> 18 -> 17 size cycle (commit 146dee7).
// So every cache here is keyed on numbers that are never reused:
//   * gen(slot)   — bumped on every (re)allocation of a slot;
//   * stamp(key)  — bumped by a builder every time it (re)writes a table's
//                   contents (a rebuild in place keeps gen, changes stamp);
// both drawn from one monotonic per-arena counter, so a value seen once never
// names another allocation or another build.  A derived table (e.g. the NTT
// pyramid of a flat twiddle table) is valid iff its memo equals
// derived_key(params, stamp(source), gen(own slot)).
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <string>

namespace qg {

template <class Backend>
struct ScratchArena {
  struct Slot {
    void* p = nullptr;
    size_t bytes = 0;
    uint64_t gen = 0;
  };
  std::map<std::string, Slot> slots;
  std::map<std::string, uint64_t> stamps;
  std::map<std::string, std::string> memo;
  uint64_t counter = 0;
  Backend backend;  // alloc / release (the device backend drains its context's streams)

  // the slot's buffer, (re)allocated when absent or smaller than `bytes`
  void* get(const std::string& slot, size_t bytes) {
    auto it = slots.find(slot);
    if (it != slots.end() && it->second.bytes >= bytes) return it->second.p;
    if (it != slots.end()) {
      backend.release(it->second.p);
      slots.erase(it);
    }
    const size_t b = bytes ? bytes : 16;
    void* p = backend.alloc(b);
    slots[slot] = Slot{p, b, ++counter};
    return p;
  }
  // generation of the slot's current allocation (0: never allocated)
  uint64_t gen(const std::string& slot) const {
    auto it = slots.find(slot);
    return it == slots.end() ? 0 : it->second.gen;
  }
  // a builder (re)wrote the contents behind `key`
  uint64_t bump(const std::string& key) { return stamps[key] = ++counter; }
  uint64_t stamp(const std::string& key) const {
    auto it = stamps.find(key);
    return it == stamps.end() ? 0 : it->second;
  }
  // the key a cached, derived table is valid under
  static std::string derived_key(const std::string& params, uint64_t src_stamp, uint64_t own_gen) {
    return params + "|s" + std::to_string(src_stamp) + "|g" + std::to_string(own_gen);
  }
  // true when memo[tag] == key (the table behind tag is valid).  A source
  // never stamped (0) is never valid.  On false the caller rebuilds and then
  // calls commit(tag, key) - only once the build's launches succeeded, so a
  // build that throws leaves the memo invalid - and a stale memo
  // is cleared here first, so a failed rebuild can never match it later.
  bool check(const std::string& tag, const std::string& key, uint64_t src_stamp = 1) {
    auto it = memo.find(tag);
    if (it == memo.end()) return false;
    if (src_stamp != 0 && it->second == key) return true;
    memo.erase(it);
    return false;
  }
  void commit(const std::string& tag, const std::string& key) { memo[tag] = key; }
  // free one slot now (no-op when absent); its generation is gone with it
  void release(const std::string& slot) {
    auto it = slots.find(slot);
    if (it == slots.end()) return;
    backend.release(it->second.p);
    slots.erase(it);
  }
  void release_all() {
    for (auto& kv : slots) backend.release(kv.second.p);
    slots.clear();
  }
};

// a small LRU of `N` slot indices keyed by a string (the S polynomial's
// w^{j(M-1)} tables per (logn, M)): slot_for returns the index holding `key`
// or the least recently used one (hit = false: the caller rebuilds it)
template <int N>
struct LruSlots {
  std::string keys[N];
  uint64_t used[N] = {};
  uint64_t tick = 0;
  int slot_for(const std::string& key, bool* hit) {
    int victim = 0;
    for (int i = 0; i < N; i++) {
      if (used[i] && keys[i] == key) {
        used[i] = ++tick;
        *hit = true;
        return i;
      }
      if (used[i] < used[victim]) victim = i;
    }
    keys[victim] = key;
    used[victim] = ++tick;
    *hit = false;
    return victim;
  }
  void forget(int i) { used[i] = 0; }
};

}  // namespace qg
