// BLAKE3 (default hash mode + XOF), host + device, and the Quill Fiat-Shamir
// transcript built on it.
//
// Replaces the `blake3` 1.8.2 crate (Cargo.lock:166-167) as used by
// transcript/src/transcript.rs:14-74:
//   new(domain):            state = B3(domain)                      :14-22
//   append_bytes(msg):      state = B3(state || msg)                :25-31
//   draw_challenge(n):      out = B3-XOF(state || "challenge")[..n]; append(out)  :48-62
//   draw_field_element():   LE(48 bytes) mod r                      :70-74
// The transcript is a 32-byte chaining state; the device copy lets the
// sumcheck round loop run without host round trips.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "field.h"

namespace qg {

#if defined(__HIPCC__) || defined(__HIP__)
#define QG_B3_CONST __device__ __constant__
#else
#define QG_B3_CONST static const
#endif

QG_HD uint32_t b3_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

QG_HD void b3_g(uint32_t* s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx;
  s[d] = b3_rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = b3_rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my;
  s[d] = b3_rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = b3_rotr(s[b] ^ s[c], 7);
}

enum : uint32_t { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };

QG_HD uint32_t b3_iv(int i) {
  switch (i) {
    case 0: return 0x6A09E667u;
    case 1: return 0xBB67AE85u;
    case 2: return 0x3C6EF372u;
    case 3: return 0xA54FF53Au;
    case 4: return 0x510E527Fu;
    case 5: return 0x9B05688Cu;
    case 6: return 0x1F83D9ABu;
    default: return 0x5BE0CD19u;
  }
}

// Full compression; out[16] receives the 16-word output state.
QG_HD void b3_compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                       uint32_t block_len, uint32_t flags, uint32_t out[16]) {
  uint32_t s[16];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = cv[i];
#pragma unroll
  for (int i = 0; i < 4; i++) s[8 + i] = b3_iv(i);
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = block[i];
#pragma unroll
  for (int r = 0; r < 7; r++) {
    b3_g(s, 0, 4, 8, 12, m[0], m[1]);
    b3_g(s, 1, 5, 9, 13, m[2], m[3]);
    b3_g(s, 2, 6, 10, 14, m[4], m[5]);
    b3_g(s, 3, 7, 11, 15, m[6], m[7]);
    b3_g(s, 0, 5, 10, 15, m[8], m[9]);
    b3_g(s, 1, 6, 11, 12, m[10], m[11]);
    b3_g(s, 2, 7, 8, 13, m[12], m[13]);
    b3_g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      // MSG_PERMUTATION = 2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8
      uint32_t p[16] = {m[2], m[6], m[3],  m[10], m[7],  m[0],  m[4],  m[13],
                        m[1], m[11], m[12], m[5], m[9], m[14], m[15], m[8]};
#pragma unroll
      for (int i = 0; i < 16; i++) m[i] = p[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[i] = s[i] ^ s[i + 8];
    out[i + 8] = s[i + 8] ^ cv[i];
  }
}

QG_HD uint32_t b3_load32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

// Streaming hasher.  STACK = depth of the chunk-CV stack: 54 covers any input
// length (host); device code uses STACK = 1, i.e. inputs of at most 2 chunks,
// which bounds its private memory (transcript messages there are < 600 B).
template <int STACK>
struct Blake3T {
  uint32_t cv[8];
  uint8_t buf[64];
  uint32_t buf_len;
  uint32_t blocks_compressed;  // within the current chunk
  uint64_t chunk_counter;
  uint32_t stack[STACK][8];
  uint32_t stack_len;

  QG_HD void init() {
#pragma unroll
    for (int i = 0; i < 8; i++) cv[i] = b3_iv(i);
    buf_len = 0;
    blocks_compressed = 0;
    chunk_counter = 0;
    stack_len = 0;
  }

  QG_HD void block_words(uint32_t w[16]) const {
    for (int i = 0; i < 16; i++) {
      uint32_t x = 0;
      for (int b = 0; b < 4; b++) {
        uint32_t idx = 4 * i + b;
        uint32_t byte = idx < buf_len ? buf[idx] : 0u;
        x |= byte << (8 * b);
      }
      w[i] = x;
    }
  }

  QG_HD void push_cv(const uint32_t new_cv[8], uint64_t total_chunks) {
    if (stack_len >= (uint32_t)STACK && (total_chunks & 1)) return;  // capacity guard
    uint32_t c[8];
    for (int i = 0; i < 8; i++) c[i] = new_cv[i];
    while ((total_chunks & 1) == 0) {
      stack_len--;
      uint32_t block[16], out[16], key[8];
      for (int i = 0; i < 8; i++) {
        block[i] = stack[stack_len][i];
        block[8 + i] = c[i];
        key[i] = b3_iv(i);
      }
      b3_compress(key, block, 0, 64, B3_PARENT, out);
      for (int i = 0; i < 8; i++) c[i] = out[i];
      total_chunks >>= 1;
    }
    for (int i = 0; i < 8; i++) stack[stack_len][i] = c[i];
    stack_len++;
  }

  QG_HD void update(const uint8_t* data, size_t len) {
    while (len > 0) {
      // chunk full (16 blocks, last one buffered): finalize chunk
      if (blocks_compressed == 15 && buf_len == 64) {
        uint32_t w[16], out[16];
        block_words(w);
        uint32_t flags = B3_CHUNK_END | (blocks_compressed == 0 ? B3_CHUNK_START : 0);
        b3_compress(cv, w, chunk_counter, 64, flags, out);
        chunk_counter++;
        push_cv(out, chunk_counter);
        for (int i = 0; i < 8; i++) cv[i] = b3_iv(i);
        blocks_compressed = 0;
        buf_len = 0;
      }
      if (buf_len == 64) {
        uint32_t w[16], out[16];
        block_words(w);
        uint32_t flags = blocks_compressed == 0 ? B3_CHUNK_START : 0;
        b3_compress(cv, w, chunk_counter, 64, flags, out);
        for (int i = 0; i < 8; i++) cv[i] = out[i];
        blocks_compressed++;
        buf_len = 0;
      }
      size_t take = 64 - buf_len;
      if (take > len) take = len;
      for (size_t i = 0; i < take; i++) buf[buf_len + i] = data[i];
      buf_len += (uint32_t)take;
      data += take;
      len -= take;
    }
  }

  // Root output node parameters -> XOF bytes
  QG_HD void finalize(uint8_t* out, size_t out_len) const {
    uint32_t in_cv[8], w[16];
    uint32_t flags = B3_CHUNK_END | (blocks_compressed == 0 ? B3_CHUNK_START : 0);
    uint64_t ctr = chunk_counter;
    uint32_t blen = buf_len;
    for (int i = 0; i < 8; i++) in_cv[i] = cv[i];
    block_words(w);
    // merge the right spine of the tree
    for (int s = (int)stack_len - 1; s >= 0; s--) {
      uint32_t o[16];
      b3_compress(in_cv, w, ctr, blen, flags, o);
      for (int i = 0; i < 8; i++) {
        w[i] = stack[s][i];
        w[8 + i] = o[i];
        in_cv[i] = b3_iv(i);
      }
      ctr = 0;
      blen = 64;
      flags = B3_PARENT;
    }
    uint64_t oc = 0;
    size_t pos = 0;
    while (pos < out_len) {
      uint32_t o[16];
      b3_compress(in_cv, w, oc, blen, flags | B3_ROOT, o);
      for (int i = 0; i < 16 && pos < out_len; i++) {
        for (int b = 0; b < 4 && pos < out_len; b++) out[pos++] = (uint8_t)(o[i] >> (8 * b));
      }
      oc++;
    }
  }
};

#if defined(__HIP_DEVICE_COMPILE__)
using Blake3 = Blake3T<1>;
#else
using Blake3 = Blake3T<54>;
#endif

// ---------------------------------------------------------------------------
// Word-oriented single-chunk BLAKE3 (input <= 1024 bytes, given as LE 32-bit
// words, tail bytes of the last word zero).  This is the device fast path of
// the transcript: no byte arrays, no private-memory buffers.
// ---------------------------------------------------------------------------
template <class Src>
QG_HD void b3_chunk_words(const Src& src, uint32_t nbytes, uint32_t* out, int nout_words) {
  uint32_t cv[8];
#pragma unroll
  for (int i = 0; i < 8; i++) cv[i] = b3_iv(i);
  const uint32_t nblocks = nbytes ? (nbytes + 63) / 64 : 1;
  for (uint32_t b = 0; b < nblocks; b++) {
    uint32_t blk[16];
    const uint32_t base = b * 16;
    const uint32_t nw = (nbytes + 3) / 4;
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = (base + i < nw) ? src(base + i) : 0u;
    const uint32_t blen = (b + 1 < nblocks) ? 64u : nbytes - b * 64;
    uint32_t flags = (b == 0 ? B3_CHUNK_START : 0u);
    if (b + 1 < nblocks) {
      uint32_t o[16];
      b3_compress(cv, blk, 0, blen, flags, o);
#pragma unroll
      for (int i = 0; i < 8; i++) cv[i] = o[i];
    } else {
      flags |= B3_CHUNK_END | B3_ROOT;
      for (int oc = 0; oc * 16 < nout_words; oc++) {
        uint32_t o[16];
        b3_compress(cv, blk, (uint64_t)oc, blen, flags, o);
        for (int i = 0; i < 16 && oc * 16 + i < nout_words; i++) out[oc * 16 + i] = o[i];
      }
    }
  }
}

struct B3ArrSrc {
  const uint32_t* p;
  QG_HD uint32_t operator()(uint32_t i) const { return p[i]; }
};

// Absorb a word message into an 8-word state: state = B3(state || msg)
QG_HD void transcript_append_words(uint32_t st[8], const uint32_t* msg, uint32_t nbytes_msg) {
  // nbytes_msg must be a multiple of 4 here
  struct Src {
    const uint32_t* s;
    const uint32_t* m;
    QG_HD uint32_t operator()(uint32_t i) const { return i < 8 ? s[i] : m[i - 8]; }
  } src{st, msg};
  uint32_t o[8];
  b3_chunk_words(src, 32 + nbytes_msg, o, 8);
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = o[i];
}

// draw_field_element on a word state (transcript.rs:48-74)
QG_HD Fr transcript_draw_fr_words(uint32_t st[8]) {
  struct Src {
    const uint32_t* s;
    QG_HD uint32_t operator()(uint32_t i) const {
      // state || "challenge" (9 bytes)
      if (i < 8) return s[i];
      if (i == 8) return 0x6c616863u;  // "chal"
      if (i == 9) return 0x676e656cu;  // "leng"
      return 0x00000065u;              // "e"
    }
  } src{st};
  uint32_t ch[12];
  b3_chunk_words(src, 41, ch, 12);
  transcript_append_words(st, ch, 48);
  Fr lo, hi;
#pragma unroll
  for (int i = 0; i < 8; i++) lo.v[i] = ch[i];
#pragma unroll
  for (int i = 0; i < 4; i++) hi.v[i] = ch[8 + i];
#pragma unroll
  for (int i = 4; i < 8; i++) hi.v[i] = 0;
  // lo may be >= r (any 256-bit value): reduce before the Montgomery product
  reduce_full<FrP>(lo.v);
  return lo * Fr::from_raw(FrP::R2) + hi * Fr::from_raw(FrP::R3);
}


#if defined(__HIPCC__) || defined(__HIP__)
// ---------------------------------------------------------------------------
// Quad-lane BLAKE3 for the device transcript's critical path.  The 4x4 state
// is split by columns over the 4 lanes of a DPP quad: lane l holds
// (v[l], v[4+l], v[8+l], v[12+l]).  The column step is one G per lane; the
// diagonal step rotates rows b, c, d by 1, 2, 3 lanes with DPP quad_perm moves
// and back.  Latency is one G chain per half-round instead of four.
// Every quad of the calling wave computes the same hash (inputs uniform).
// ---------------------------------------------------------------------------
struct B3Sched {
  int s[7][16];
};

constexpr B3Sched b3_make_sched() {
  B3Sched r{};
  const int perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  for (int i = 0; i < 16; i++) r.s[0][i] = i;
  for (int k = 1; k < 7; k++)
    for (int i = 0; i < 16; i++) r.s[k][i] = r.s[k - 1][perm[i]];
  return r;
}

// word for lane l of a quad: (w0, w1, w2, w3)[l]   (l uniform per lane)
QG_DEV uint32_t b3_pick4(uint32_t l, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  const uint32_t lo = (l & 1) ? w1 : w0, hi = (l & 1) ? w3 : w2;
  return (l & 2) ? hi : lo;
}

template <int CTRL>
QG_DEV uint32_t b3_qperm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}

QG_DEV void b3_g1(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t mx, uint32_t my) {
  a = a + b + mx;
  d = b3_rotr(d ^ a, 16);
  c = c + d;
  b = b3_rotr(b ^ c, 12);
  a = a + b + my;
  d = b3_rotr(d ^ a, 8);
  c = c + d;
  b = b3_rotr(b ^ c, 7);
}

// One compression.  cvl/cvh: this lane's chaining words cv[l], cv[4+l];
// m: the (uniform) 16 message words.  Returns this lane's output words
// o0 = out[l], o1 = out[4+l], o2 = out[8+l], o3 = out[12+l].
QG_DEV void b3_compress_quad(uint32_t l, uint32_t cvl, uint32_t cvh, const uint32_t (&m)[16],
                             uint64_t counter, uint32_t blen, uint32_t flags, uint32_t& o0,
                             uint32_t& o1, uint32_t& o2, uint32_t& o3) {
  constexpr B3Sched S = b3_make_sched();
  uint32_t a = cvl, b = cvh;
  uint32_t c = b3_pick4(l, 0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au);
  uint32_t d = b3_pick4(l, (uint32_t)counter, (uint32_t)(counter >> 32), blen, flags);
#pragma unroll
  for (int r = 0; r < 7; r++) {
    b3_g1(a, b, c, d, b3_pick4(l, m[S.s[r][0]], m[S.s[r][2]], m[S.s[r][4]], m[S.s[r][6]]),
          b3_pick4(l, m[S.s[r][1]], m[S.s[r][3]], m[S.s[r][5]], m[S.s[r][7]]));
    // diagonalize: b <- lane l+1, c <- lane l+2, d <- lane l+3 (mod 4)
    b = b3_qperm<0x39>(b);
    c = b3_qperm<0x4E>(c);
    d = b3_qperm<0x93>(d);
    b3_g1(a, b, c, d, b3_pick4(l, m[S.s[r][8]], m[S.s[r][10]], m[S.s[r][12]], m[S.s[r][14]]),
          b3_pick4(l, m[S.s[r][9]], m[S.s[r][11]], m[S.s[r][13]], m[S.s[r][15]]));
    b = b3_qperm<0x93>(b);
    c = b3_qperm<0x4E>(c);
    d = b3_qperm<0x39>(d);
  }
  o0 = a ^ c;
  o1 = b ^ d;
  o2 = c ^ cvl;
  o3 = d ^ cvh;
}

// BLAKE3 of a word message in LDS (<= 1024 bytes; bytes past nbytes up to the
// next 64-byte boundary must be zero), root output words [0, nout) (nout <= 16)
// written to out (LDS or global) by lanes 0..3.  Call with the whole wave.
QG_DEV void b3_hash_quad(const uint32_t* msg, uint32_t nbytes, uint32_t* out, int nout) {
  const uint32_t lane = __lane_id(), l = lane & 3;
  uint32_t cvl = b3_pick4(l, 0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au);
  uint32_t cvh = b3_pick4(l, 0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u);
  const uint32_t nblocks = nbytes ? (nbytes + 63) / 64 : 1;
  for (uint32_t bi = 0; bi < nblocks; bi++) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = msg[bi * 16 + i];
    const bool last = bi + 1 == nblocks;
    const uint32_t blen = last ? nbytes - bi * 64 : 64u;
    const uint32_t flags = (bi == 0 ? B3_CHUNK_START : 0u) | (last ? (B3_CHUNK_END | B3_ROOT) : 0u);
    uint32_t o0, o1, o2, o3;
    b3_compress_quad(l, cvl, cvh, m, 0, blen, flags, o0, o1, o2, o3);
    if (!last) {
      cvl = o0;
      cvh = o1;
    } else if (lane < 4) {
      if ((int)l < nout) out[l] = o0;
      if ((int)(4 + l) < nout) out[4 + l] = o1;
      if ((int)(8 + l) < nout) out[8 + l] = o2;
      if ((int)(12 + l) < nout) out[12 + l] = o3;
    }
  }
}
#endif

// ---------------------------------------------------------------------------
// Transcript primitives over a 32-byte state
// ---------------------------------------------------------------------------
QG_HD void transcript_init(uint8_t state[32], const uint8_t* domain, size_t len) {
  Blake3 h;
  h.init();
  h.update(domain, len);
  h.finalize(state, 32);
}

QG_HD void transcript_append(uint8_t state[32], const uint8_t* msg, size_t len) {
  Blake3 h;
  h.init();
  h.update(state, 32);
  h.update(msg, len);
  h.finalize(state, 32);
}

// n <= 64 bytes of challenge; re-absorbs them (transcript.rs:48-62)
QG_HD void transcript_draw(uint8_t state[32], uint8_t* out, size_t n) {
  Blake3 h;
  h.init();
  h.update(state, 32);
  const uint8_t label[9] = {'c', 'h', 'a', 'l', 'l', 'e', 'n', 'g', 'e'};
  h.update(label, 9);
  h.finalize(out, n);
  transcript_append(state, out, n);
}

// 48 LE bytes -> Fr (Montgomery), == from_le_bytes_mod_order (transcript.rs:70-74)
QG_HD Fr fr_from_le48(const uint8_t b[48]) {
  Fr lo, hi;
  for (int i = 0; i < 8; i++) lo.v[i] = b3_load32(b + 4 * i);
  for (int i = 0; i < 4; i++) hi.v[i] = b3_load32(b + 32 + 4 * i);
  for (int i = 4; i < 8; i++) hi.v[i] = 0;
  // lo*R^2*R^-1 = lo*R ; hi*R^3*R^-1 = hi*R^2 = (hi*2^256)*R
  // lo may be >= r (any 256-bit value): reduce before the Montgomery product
  reduce_full<FrP>(lo.v);
  return lo * Fr::from_raw(FrP::R2) + hi * Fr::from_raw(FrP::R3);
}

QG_HD Fr transcript_draw_fr(uint8_t state[32]) {
  uint8_t b[48];
  transcript_draw(state, b, 48);
  return fr_from_le48(b);
}

// Fr (Montgomery) -> 32 canonical LE bytes
QG_HD void fr_to_bytes(const Fr& x, uint8_t* out) {
  Fr c = from_mont(x);
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(c.v[i] >> (8 * b));
}

QG_HD void u64_to_bytes(uint64_t v, uint8_t* out) {
  for (int b = 0; b < 8; b++) out[b] = (uint8_t)(v >> (8 * b));
}

}  // namespace qg
