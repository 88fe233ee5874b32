// CPU check of the scratch arena's generation rule (quill-zkvm_amd/csrc/arena.h)
// with a malloc backend that deliberately hands a freed address back, the way
// hipMalloc does after scratch regrowth.  Prints "ok <name>" per check; exits
// non-zero on the first failure.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../quill-zkvm_amd/csrc/arena.h"

// allocator that reuses the most recently freed block when it is big enough
struct ReuseAlloc {
  static std::vector<std::pair<void*, size_t>>& freed() {
    static std::vector<std::pair<void*, size_t>> f;
    return f;
  }
  static std::vector<std::pair<void*, size_t>>& live() {
    static std::vector<std::pair<void*, size_t>> l;
    return l;
  }
  static void* alloc(size_t b) {
    auto& f = freed();
    for (size_t i = f.size(); i-- > 0;)
      if (f[i].second >= b) {
        void* p = f[i].first;
        live().push_back(f[i]);
        f.erase(f.begin() + (long)i);
        return p;
      }
    void* p = malloc(b < 4096 ? 4096 : b);
    live().push_back({p, b < 4096 ? 4096 : b});
    return p;
  }
  static void release(void* p) {
    auto& l = live();
    for (size_t i = 0; i < l.size(); i++)
      if (l[i].first == p) {
        freed().push_back(l[i]);
        l.erase(l.begin() + (long)i);
        return;
      }
  }
};

static int fails = 0;
#define CHECK(name, cond)                    \
  do {                                       \
    if (cond) {                              \
      printf("ok %s\n", name);               \
    } else {                                 \
      printf("FAIL %s\n", name);             \
      fails++;                               \
    }                                        \
  } while (0)

using Arena = qg::ScratchArena<ReuseAlloc>;

// a derived table of source slot `src` (the NTT pyramid's rule); returns true
// when it had to be rebuilt
static bool derived(Arena& a, const std::string& src, int logn) {
  const std::string tag = "pyr:" + src;
  a.get(tag, (size_t)1 << logn);
  const uint64_t st = a.stamp(src);
  const std::string key = Arena::derived_key(std::to_string(logn), st, a.gen(tag));
  if (a.check(tag, key, st)) return false;
  a.commit(tag, key);
  return true;
}

// a flat table build (ntt_twiddles' rule): rebuilds and stamps when the
// (logn, generation) key changes
static bool build_flat(Arena& a, const std::string& slot, int logn) {
  a.get(slot, (size_t)1 << logn);
  const std::string key = std::to_string(logn) + "|g" + std::to_string(a.gen(slot));
  if (a.check(slot, key)) return false;
  a.bump(slot);
  a.commit(slot, key);
  return true;
}

int main() {
  Arena a;
  // 1. a slot that fits keeps its buffer and generation; growth re-allocates
  void* p1 = a.get("x", 100);
  const uint64_t g1 = a.gen("x");
  CHECK("fit_keeps_gen", a.get("x", 50) == p1 && a.gen("x") == g1);
  a.get("x", 1 << 20);
  const uint64_t g2 = a.gen("x");
  CHECK("grow_new_gen", g2 > g1);
  CHECK("unknown_slot_gen0", a.gen("never") == 0 && a.stamp("never") == 0);

  // 2. a freed address handed to another slot carries a different generation
  Arena b;
  void* q1 = b.get("old", 1 << 16);
  const uint64_t qg1 = b.gen("old");
  b.get("old", 1 << 18);  // frees q1
  void* q2 = b.get("other", 1 << 16);
  CHECK("address_reused_by_backend", q2 == q1);
  CHECK("reused_address_new_gen", b.gen("other") != qg1 && b.gen("other") > b.gen("old"));

  // 3. the 17 -> 18 -> 17 size cycle that served a stale pyramid (146dee7):
  //    forward / inverse flat tables regrow, addresses swap, every derived
  //    table must be rebuilt after each flat rebuild and reused otherwise
  Arena c;
  CHECK("flat_first_build", build_flat(c, "tw", 17) && build_flat(c, "twi", 17));
  CHECK("derived_first_build", derived(c, "tw", 17) && derived(c, "twi", 17));
  CHECK("derived_reused", !derived(c, "tw", 17) && !derived(c, "twi", 17));
  CHECK("flat_reused", !build_flat(c, "tw", 17));
  CHECK("flat_regrow_18", build_flat(c, "tw", 18) && build_flat(c, "twi", 18));
  CHECK("derived_rebuilt_18", derived(c, "tw", 18) && derived(c, "twi", 18));
  // back to 17: the 18 tables fit, so the slots keep their buffers, but the
  // builds change the contents: the stamp must force the derived rebuild even
  // though every address and allocation generation is unchanged
  const uint64_t gtw = c.gen("tw");
  CHECK("flat_rebuild_in_place_17", build_flat(c, "tw", 17) && c.gen("tw") == gtw);
  build_flat(c, "twi", 17);
  CHECK("derived_rebuilt_after_in_place", derived(c, "tw", 17) && derived(c, "twi", 17));
  CHECK("derived_stable_again", !derived(c, "tw", 17));

  // 4. a derived table of a never-built source is never valid
  Arena d;
  CHECK("unstamped_source_invalid", derived(d, "nobody", 4) && derived(d, "nobody", 4));

  // 5. the (logn, M) LRU of the S polynomial's w^{j(M-1)} tables
  qg::LruSlots<4> lru;
  bool hit = true;
  const int s0 = lru.slot_for("17:65536", &hit);
  CHECK("lru_first_miss", !hit);
  const int s1 = lru.slot_for("18:131072", &hit);
  CHECK("lru_second_miss_other_slot", !hit && s1 != s0);
  CHECK("lru_hit", lru.slot_for("17:65536", &hit) == s0 && hit);
  lru.slot_for("a", &hit);
  lru.slot_for("b", &hit);
  const int s5 = lru.slot_for("c", &hit);  // evicts the least recent: 18:131072
  CHECK("lru_evicts_least_recent", !hit && s5 == s1);
  CHECK("lru_recent_kept", lru.slot_for("17:65536", &hit) == s0 && hit);
  // two alternating keys never evict each other (the hash % 4 slots could)
  int rebuilds = 0;
  qg::LruSlots<4> l2;
  for (int i = 0; i < 20; i++) {
    l2.slot_for(i & 1 ? "23:4194304" : "22:2097152", &hit);
    rebuilds += !hit;
  }
  CHECK("lru_alternating_two_builds", rebuilds == 2);

  // 6. check + commit: a build whose launches throw never
  //    commits, so the table stays invalid; a mismatching check clears the
  //    stale memo, so a later failed rebuild cannot revive the old key
  Arena e;
  CHECK("no_memo_invalid", !e.check("t", "k1"));
  CHECK("uncommitted_build_stays_invalid", !e.check("t", "k1"));
  e.commit("t", "k1");
  CHECK("committed_valid", e.check("t", "k1"));
  CHECK("other_key_invalid", !e.check("t", "k2"));
  CHECK("stale_memo_cleared", !e.check("t", "k1"));

  a.release_all();
  b.release_all();
  c.release_all();
  d.release_all();
  return fails ? 1 : 0;
}
