// Virtual-polynomial expression compiler (host side), shared by the sumcheck
// and the Logup column kernels.  The postfix program (qg_expr_op, the
// reference's VirtualPolyExpr tree of virtual_polynomial.rs:9-37 flattened) is
// expanded into a sum of monomials: coefficient x product of table entries.
#pragma once
#include <algorithm>
#include <map>
#include <vector>

#include "common.h"

namespace qg {

// ---------------------------------------------------------------- programs
struct Mono {
  std::vector<uint32_t> fac;  // sorted input indices (with multiplicity)
  Fr coeff;
};

struct SopProgram {
  std::vector<uint32_t> used;    // original table index of each compact slot
  std::vector<uint32_t> mono_len;
  std::vector<uint32_t> fac;     // compact slot indices
  std::vector<Fr> coeff;
  std::vector<uint8_t> is_one;
  uint32_t degree = 0;           // max monomial degree
};

typedef std::map<std::vector<uint32_t>, Fr> PolyMap;

inline PolyMap pm_add(const PolyMap& a, const PolyMap& b) {
  PolyMap r = a;
  for (auto& kv : b) {
    auto it = r.find(kv.first);
    if (it == r.end()) r[kv.first] = kv.second;
    else it->second = it->second + kv.second;
  }
  return r;
}

inline PolyMap pm_mul(const PolyMap& a, const PolyMap& b, size_t cap) {
  PolyMap r;
  for (auto& x : a)
    for (auto& y : b) {
      std::vector<uint32_t> f = x.first;
      f.insert(f.end(), y.first.begin(), y.first.end());
      std::sort(f.begin(), f.end());
      Fr c = x.second * y.second;
      auto it = r.find(f);
      if (it == r.end()) r[f] = c;
      else it->second = it->second + c;
      QG_CHECK(r.size() <= cap, QG_ERR_UNSUPPORTED, "expression expands to too many monomials");
    }
  return r;
}

// syntactic degree (Mul adds, Add maxes, Input 1, Const 0) — sizes the outputs
inline uint32_t expr_degree(const qg_expr_op* prog, size_t len) {
  std::vector<uint32_t> st;
  for (size_t i = 0; i < len; i++) {
    const uint32_t op = prog[i].op;
    if (op == QG_OP_INPUT) st.push_back(1);
    else if (op == QG_OP_CONST) st.push_back(0);
    else if (op == QG_OP_ADD || op == QG_OP_MUL) {
      QG_CHECK(st.size() >= 2, QG_ERR_INVALID, "malformed expression (stack underflow)");
      uint32_t b = st.back();
      st.pop_back();
      uint32_t a = st.back();
      st.pop_back();
      st.push_back(op == QG_OP_ADD ? std::max(a, b) : a + b);
    } else {
      throw Error(QG_ERR_INVALID, "unknown expression opcode");
    }
  }
  QG_CHECK(st.size() == 1, QG_ERR_INVALID, "malformed expression (stack size != 1)");
  return st[0];
}

inline SopProgram compile_program(const qg_expr_op* prog, size_t len, const uint64_t* consts,
                                  size_t nconsts, uint32_t ntables) {
  std::vector<PolyMap> st;
  const size_t cap = 1024;
  for (size_t i = 0; i < len; i++) {
    const uint32_t op = prog[i].op, arg = prog[i].arg;
    if (op == QG_OP_INPUT) {
      QG_CHECK(arg < ntables, QG_ERR_INVALID, "expression input index out of range");
      PolyMap m;
      m[{arg}] = Fr::one();
      st.push_back(m);
    } else if (op == QG_OP_CONST) {
      QG_CHECK(arg < nconsts, QG_ERR_INVALID, "expression constant index out of range");
      PolyMap m;
      m[{}] = fr_import(consts + 4 * (size_t)arg);
      st.push_back(m);
    } else if (op == QG_OP_ADD || op == QG_OP_MUL) {
      QG_CHECK(st.size() >= 2, QG_ERR_INVALID, "malformed expression (stack underflow)");
      PolyMap b = st.back();
      st.pop_back();
      PolyMap a = st.back();
      st.pop_back();
      st.push_back(op == QG_OP_ADD ? pm_add(a, b) : pm_mul(a, b, cap));
    } else {
      throw Error(QG_ERR_INVALID, "unknown expression opcode");
    }
  }
  QG_CHECK(st.size() == 1, QG_ERR_INVALID, "malformed expression (stack size != 1)");
  SopProgram sp;
  std::map<uint32_t, uint32_t> slot;
  for (auto& kv : st[0]) {
    if (kv.second.is_zero()) continue;
    for (uint32_t t : kv.first)
      if (!slot.count(t)) slot[t] = 0;
  }
  for (auto& kv : slot) {
    kv.second = (uint32_t)sp.used.size();
    sp.used.push_back(kv.first);
  }
  for (auto& kv : st[0]) {
    if (kv.second.is_zero()) continue;
    sp.mono_len.push_back((uint32_t)kv.first.size());
    for (uint32_t t : kv.first) sp.fac.push_back(slot[t]);
    sp.coeff.push_back(kv.second);
    sp.is_one.push_back(kv.second == Fr::one() ? 1 : 0);
    sp.degree = std::max<uint32_t>(sp.degree, (uint32_t)kv.first.size());
  }
  return sp;
}

}  // namespace qg
