// Device-side interpreter for the predicate / projection programs of plan.h.
//
// Value semantics follow Siddhi's expression executors on Java primitives
// (SURVEY.md App. A.2): int/long arithmetic wraps, int division truncates,
// `%` takes the dividend's sign, int/long division or remainder by zero
// yields null, a comparison with a null operand is false, float ops are
// IEEE binary32, double ops IEEE binary64, NaN compares false.
//
// The register file lives in LDS laid out [reg][thread] (64 consecutive lanes
// touch 64 consecutive 8-byte words: conflict-free ds_read_b64 / ds_write_b64),
// so programs with runtime register operands never spill to scratch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace cep {

__device__ __forceinline__ float as_f32(uint64_t v) { return __uint_as_float((uint32_t)v); }
__device__ __forceinline__ double as_f64(uint64_t v) { return __longlong_as_double((long long)v); }
__device__ __forceinline__ uint64_t from_f32(float f) { return (uint64_t)__float_as_uint(f); }
__device__ __forceinline__ uint64_t from_f64(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ uint64_t from_i32(int32_t i) { return (uint64_t)(int64_t)i; }

// Load one element of a typed column as a VM word.
__device__ __forceinline__ uint64_t load_col(const void* p, int type, int64_t row) {
  switch (type) {
    case T_LONG:
    case T_DOUBLE:
      return ((const uint64_t*)p)[row];
    case T_BOOL:
      return ((const uint8_t*)p)[row] ? 1u : 0u;
    case T_FLOAT:
      return (uint64_t)((const uint32_t*)p)[row];
    default:  // INT, STRING (dictionary id)
      return from_i32(((const int32_t*)p)[row]);
  }
}

__device__ __forceinline__ void store_col(void* p, int type, int64_t row, uint64_t v) {
  switch (type) {
    case T_LONG:
    case T_DOUBLE:
      ((uint64_t*)p)[row] = v;
      break;
    case T_BOOL:
      ((uint8_t*)p)[row] = (uint8_t)(v & 1);
      break;
    default:
      ((uint32_t*)p)[row] = (uint32_t)v;
      break;
  }
}

__device__ __forceinline__ uint64_t vm_convert(uint64_t v, int from, int to) {
  if (from == to) return v;
  if (to == T_LONG) return v;  // int words are already sign-extended
  if (to == T_FLOAT) {
    if (from == T_INT) return from_f32((float)(int32_t)v);
    if (from == T_LONG) return from_f32((float)(int64_t)v);
    return v;
  }
  if (to == T_DOUBLE) {
    if (from == T_INT) return from_f64((double)(int32_t)v);
    if (from == T_LONG) return from_f64((double)(int64_t)v);
    if (from == T_FLOAT) return from_f64((double)as_f32(v));
  }
  return v;
}

// Arithmetic; returns false when the result is null (int div/mod by zero).
__device__ __forceinline__ bool vm_arith(int op, int t, uint64_t a, uint64_t b, uint64_t* r) {
  switch (t) {
    case T_INT: {
      int32_t x = (int32_t)a, y = (int32_t)b;
      uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
      int32_t z;
      switch (op) {
        case OP_ADD: z = (int32_t)(ux + uy); break;
        case OP_SUB: z = (int32_t)(ux - uy); break;
        case OP_MUL: z = (int32_t)(ux * uy); break;
        case OP_DIV:
          if (y == 0) return false;
          z = (y == -1) ? (int32_t)(0u - ux) : x / y;
          break;
        default:
          if (y == 0) return false;
          z = (y == -1) ? 0 : x % y;
          break;
      }
      *r = from_i32(z);
      return true;
    }
    case T_LONG: {
      int64_t x = (int64_t)a, y = (int64_t)b;
      uint64_t z;
      switch (op) {
        case OP_ADD: z = a + b; break;
        case OP_SUB: z = a - b; break;
        case OP_MUL: z = a * b; break;
        case OP_DIV:
          if (y == 0) return false;
          z = (y == -1) ? (0ull - a) : (uint64_t)(x / y);
          break;
        default:
          if (y == 0) return false;
          z = (y == -1) ? 0ull : (uint64_t)(x % y);
          break;
      }
      *r = z;
      return true;
    }
    case T_FLOAT: {
      float x = as_f32(a), y = as_f32(b), z;
      switch (op) {
        case OP_ADD: z = x + y; break;
        case OP_SUB: z = x - y; break;
        case OP_MUL: z = x * y; break;
        case OP_DIV: z = x / y; break;
        default: z = fmodf(x, y); break;
      }
      *r = from_f32(z);
      return true;
    }
    default: {
      double x = as_f64(a), y = as_f64(b), z;
      switch (op) {
        case OP_ADD: z = x + y; break;
        case OP_SUB: z = x - y; break;
        case OP_MUL: z = x * y; break;
        case OP_DIV: z = x / y; break;
        default: z = fmod(x, y); break;
      }
      *r = from_f64(z);
      return true;
    }
  }
}

__device__ __forceinline__ bool vm_compare(int op, int t, uint64_t a, uint64_t b) {
  switch (t) {
    case T_LONG: {
      int64_t x = (int64_t)a, y = (int64_t)b;
      switch (op) {
        case OP_EQ: return x == y;
        case OP_NE: return x != y;
        case OP_LT: return x < y;
        case OP_LE: return x <= y;
        case OP_GT: return x > y;
        default: return x >= y;
      }
    }
    case T_FLOAT: {
      float x = as_f32(a), y = as_f32(b);
      switch (op) {
        case OP_EQ: return x == y;
        case OP_NE: return x != y;
        case OP_LT: return x < y;
        case OP_LE: return x <= y;
        case OP_GT: return x > y;
        default: return x >= y;
      }
    }
    case T_DOUBLE: {
      double x = as_f64(a), y = as_f64(b);
      switch (op) {
        case OP_EQ: return x == y;
        case OP_NE: return x != y;
        case OP_LT: return x < y;
        case OP_LE: return x <= y;
        case OP_GT: return x > y;
        default: return x >= y;
      }
    }
    default: {  // INT, BOOL, STRING ids
      int32_t x = (int32_t)a, y = (int32_t)b;
      switch (op) {
        case OP_EQ: return x == y;
        case OP_NE: return x != y;
        case OP_LT: return x < y;
        case OP_LE: return x <= y;
        case OP_GT: return x > y;
        default: return x >= y;
      }
    }
  }
}

// Evaluate program at `off`.  `R` is this block's LDS register file, `lane`
// the thread's column in it, `stride` the block size.  Env supplies
// col(c, type), cap(i), outv(i), agg(i), ts().  Returns the result word of
// register 0; *is_null reports a null result.
template <class Env>
__device__ __forceinline__ uint64_t vm_eval(const Ins* __restrict__ code,
                                            const uint64_t* __restrict__ konst, int off,
                                            uint64_t* R, int lane, int stride,
                                            const Env& env, bool* is_null) {
  uint32_t nullm = 0;
#define VREG(r) R[(r) * stride + lane]
  for (int pc = off;; ++pc) {
    const Ins in = code[pc];
    const int d = in.dst, a = in.a, b = in.b;
    switch (in.op) {
      case OP_END:
        *is_null = (nullm & 1u) != 0;
        return VREG(0);
      case OP_LDCOL:
        VREG(d) = env.col((int)in.imm, b);
        nullm &= ~(1u << d);
        break;
      case OP_LDTS:
        VREG(d) = (uint64_t)env.ts();
        nullm &= ~(1u << d);
        break;
      case OP_LDK:
        VREG(d) = konst[in.imm];
        nullm &= ~(1u << d);
        break;
      case OP_LDCAP:
        VREG(d) = env.cap((int)in.imm);
        nullm &= ~(1u << d);
        break;
      case OP_LDOUT: {
        bool n = false;
        VREG(d) = env.outv((int)in.imm, &n);
        nullm = n ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
      }
      case OP_LDAGG: {
        bool n = false;
        VREG(d) = env.agg((int)in.imm, &n);
        nullm = n ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
      }
      case OP_CVT:
        VREG(d) = vm_convert(VREG(a), (int)(in.imm >> 8), (int)(in.imm & 0xff));
        nullm = (nullm & (1u << a)) ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
      case OP_ADD:
      case OP_SUB:
      case OP_MUL:
      case OP_DIV:
      case OP_MOD: {
        uint64_t r = 0;
        bool nn = ((nullm >> a) | (nullm >> b)) & 1u;
        if (!nn) nn = !vm_arith(in.op, (int)in.imm, VREG(a), VREG(b), &r);
        VREG(d) = r;
        nullm = nn ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
      }
      case OP_NEG: {
        uint64_t v = VREG(a), r;
        switch ((int)in.imm) {
          case T_INT: r = from_i32((int32_t)(0u - (uint32_t)v)); break;
          case T_LONG: r = 0ull - v; break;
          case T_FLOAT: r = from_f32(-as_f32(v)); break;
          default: r = from_f64(-as_f64(v)); break;
        }
        VREG(d) = r;
        nullm = (nullm & (1u << a)) ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
      }
      case OP_EQ:
      case OP_NE:
      case OP_LT:
      case OP_LE:
      case OP_GT:
      case OP_GE: {
        bool nn = ((nullm >> a) | (nullm >> b)) & 1u;
        VREG(d) = (!nn && vm_compare(in.op, (int)in.imm, VREG(a), VREG(b))) ? 1u : 0u;
        nullm &= ~(1u << d);
        break;
      }
      case OP_AND:
        VREG(d) = ((VREG(a) & 1u) && !((nullm >> a) & 1u) && (VREG(b) & 1u) &&
                   !((nullm >> b) & 1u)) ? 1u : 0u;
        nullm &= ~(1u << d);
        break;
      case OP_OR:
        VREG(d) = (((VREG(a) & 1u) && !((nullm >> a) & 1u)) ||
                   ((VREG(b) & 1u) && !((nullm >> b) & 1u))) ? 1u : 0u;
        nullm &= ~(1u << d);
        break;
      case OP_NOT:
        VREG(d) = ((VREG(a) & 1u) && !((nullm >> a) & 1u)) ? 0u : 1u;
        nullm &= ~(1u << d);
        break;
      default:  // OP_MOV
        VREG(d) = VREG(a);
        nullm = (nullm & (1u << a)) ? (nullm | (1u << d)) : (nullm & ~(1u << d));
        break;
    }
  }
#undef VREG
}

}  // namespace cep

namespace cep {

// ---- global-address-space vector loads (avoid flat_load on generic pointers)
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload4(const void* p) {
  const v4u32 x = *(const __attribute__((address_space(1))) v4u32*)p;
  return make_uint4(x.x, x.y, x.z, x.w);
}

// ---- stage-wise evaluation of one predicate term over N rows ---------------
// Each stage switches once on the (uniform) type / operator and then runs a
// straight loop over the N values, instead of switching per element.
template <int N>
__device__ __forceinline__ void convert_run(uint64_t (&v)[N], int from, int to) {
  if (from == to || to == T_LONG) return;
  if (to == T_FLOAT) {
    if (from == T_INT) {
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = from_f32((float)(int32_t)v[e]);
    } else if (from == T_LONG) {
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = from_f32((float)(int64_t)v[e]);
    }
  } else if (to == T_DOUBLE) {
    if (from == T_INT) {
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = from_f64((double)(int32_t)v[e]);
    } else if (from == T_LONG) {
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = from_f64((double)(int64_t)v[e]);
    } else if (from == T_FLOAT) {
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = from_f64((double)as_f32(v[e]));
    }
  }
}

#define CEP_RUN(expr)                     \
  _Pragma("unroll") for (int e = 0; e < N; ++e) { expr; }

// Unsigned 32-bit division by an invariant divisor d >= 1 (Granlund-
// Montgomery / "round-up" magic): l = ceil(log2 d), m = floor(2^32 (2^l - d)
// / d) + 1, n / d = (t + ((n - t) >> 1)) >> (l - 1) with t = mulhi(m, n);
// exact for every 32-bit n (checked exhaustively over edge and random
// dividends / divisors).  d = 1 is the identity.
struct Div32 {
  uint32_t m;
  int l;
};
__device__ __forceinline__ Div32 div32_magic(uint32_t d) {
  Div32 r{0u, 0};
  if (d > 1) {
    r.l = 32 - __builtin_clz(d - 1u);
    r.m = (uint32_t)(((((uint64_t)1 << r.l) - d) << 32) / d) + 1u;
  }
  return r;
}
__device__ __forceinline__ uint32_t div32_apply(uint32_t n, uint32_t d, const Div32& dm) {
  if (d == 1u) return n;
  const uint32_t t = __umulhi(dm.m, n);
  return (t + ((n - t) >> 1)) >> (dm.l - 1);
}

template <int N>
__device__ __forceinline__ void arith_run(uint64_t (&v)[N], int op, int t, uint64_t k,
                                          uint32_t* nullm) {
  switch (t) {
    case T_INT: {
      const int32_t y = (int32_t)k;
      switch (op) {
        case OP_ADD: CEP_RUN(v[e] = from_i32((int32_t)((uint32_t)v[e] + (uint32_t)y))) break;
        case OP_SUB: CEP_RUN(v[e] = from_i32((int32_t)((uint32_t)v[e] - (uint32_t)y))) break;
        case OP_MUL: CEP_RUN(v[e] = from_i32((int32_t)((uint32_t)v[e] * (uint32_t)y))) break;
        case OP_DIV:
        default: {   // OP_MOD
          if (y == 0) { *nullm = ~0u; return; }
          if (y == -1) {
            if (op == OP_DIV) { CEP_RUN(v[e] = from_i32((int32_t)(0u - (uint32_t)v[e]))) }
            else { CEP_RUN(v[e] = 0) }
            return;
          }
          // truncated division by a constant (Java int / and %): |x| / |y| by
          // magic-number multiplication (one mul_hi, exact for every 32-bit
          // dividend), then the signs — not a division routine per row
          const uint32_t d = y < 0 ? 0u - (uint32_t)y : (uint32_t)y;
          const Div32 dm = div32_magic(d);
          CEP_RUN({
            const int32_t x = (int32_t)v[e];
            const uint32_t n = x < 0 ? 0u - (uint32_t)x : (uint32_t)x;
            const uint32_t q = div32_apply(n, d, dm);
            if (op == OP_DIV) v[e] = from_i32((int32_t)(((x < 0) != (y < 0)) ? 0u - q : q));
            else {
              const uint32_t r = n - q * d;
              v[e] = from_i32((int32_t)(x < 0 ? 0u - r : r));
            }
          })
          break;
        }
      }
      return;
    }
    case T_LONG: {
      const int64_t y = (int64_t)k;
      switch (op) {
        case OP_ADD: CEP_RUN(v[e] = v[e] + k) break;
        case OP_SUB: CEP_RUN(v[e] = v[e] - k) break;
        case OP_MUL: CEP_RUN(v[e] = v[e] * k) break;
        case OP_DIV:
          if (y == 0) { *nullm = ~0u; return; }
          if (y == -1) { CEP_RUN(v[e] = 0ull - v[e]) }
          else { CEP_RUN(v[e] = (uint64_t)((int64_t)v[e] / y)) }
          break;
        default:
          if (y == 0) { *nullm = ~0u; return; }
          if (y == -1) { CEP_RUN(v[e] = 0) }
          else { CEP_RUN(v[e] = (uint64_t)((int64_t)v[e] % y)) }
          break;
      }
      return;
    }
    case T_FLOAT: {
      const float y = as_f32(k);
      switch (op) {
        case OP_ADD: CEP_RUN(v[e] = from_f32(as_f32(v[e]) + y)) break;
        case OP_SUB: CEP_RUN(v[e] = from_f32(as_f32(v[e]) - y)) break;
        case OP_MUL: CEP_RUN(v[e] = from_f32(as_f32(v[e]) * y)) break;
        case OP_DIV: CEP_RUN(v[e] = from_f32(as_f32(v[e]) / y)) break;
        default: CEP_RUN(v[e] = from_f32(fmodf(as_f32(v[e]), y))) break;
      }
      return;
    }
    default: {
      const double y = as_f64(k);
      switch (op) {
        case OP_ADD: CEP_RUN(v[e] = from_f64(as_f64(v[e]) + y)) break;
        case OP_SUB: CEP_RUN(v[e] = from_f64(as_f64(v[e]) - y)) break;
        case OP_MUL: CEP_RUN(v[e] = from_f64(as_f64(v[e]) * y)) break;
        case OP_DIV: CEP_RUN(v[e] = from_f64(as_f64(v[e]) / y)) break;
        default: CEP_RUN(v[e] = from_f64(fmod(as_f64(v[e]), y))) break;
      }
      return;
    }
  }
}

template <int N, class T>
__device__ __forceinline__ uint32_t cmp_run_t(const T (&x)[N], int op, T y) {
  uint32_t b = 0;
  switch (op) {
    case OP_EQ: CEP_RUN(b |= (x[e] == y ? 1u : 0u) << e) break;
    case OP_NE: CEP_RUN(b |= (x[e] != y ? 1u : 0u) << e) break;
    case OP_LT: CEP_RUN(b |= (x[e] < y ? 1u : 0u) << e) break;
    case OP_LE: CEP_RUN(b |= (x[e] <= y ? 1u : 0u) << e) break;
    case OP_GT: CEP_RUN(b |= (x[e] > y ? 1u : 0u) << e) break;
    default: CEP_RUN(b |= (x[e] >= y ? 1u : 0u) << e) break;
  }
  return b;
}

template <int N>
__device__ __forceinline__ uint32_t compare_run(const uint64_t (&v)[N], int op, int t, uint64_t k) {
  switch (t) {
    case T_LONG: {
      int64_t x[N];
      CEP_RUN(x[e] = (int64_t)v[e])
      return cmp_run_t<N, int64_t>(x, op, (int64_t)k);
    }
    case T_FLOAT: {
      float x[N];
      CEP_RUN(x[e] = as_f32(v[e]))
      return cmp_run_t<N, float>(x, op, as_f32(k));
    }
    case T_DOUBLE: {
      double x[N];
      CEP_RUN(x[e] = as_f64(v[e]))
      return cmp_run_t<N, double>(x, op, as_f64(k));
    }
    default: {
      int32_t x[N];
      CEP_RUN(x[e] = (int32_t)v[e])
      return cmp_run_t<N, int32_t>(x, op, (int32_t)k);
    }
  }
}
#undef CEP_RUN

}  // namespace cep
