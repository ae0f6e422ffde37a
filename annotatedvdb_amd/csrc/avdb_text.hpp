// Text helpers shared by the VCF tokenizer (K0, avdb_vcf.hip) and the COPY /
// .mapping formatter (K5, avdb_format.hip).
#pragma once

#include "avdb_internal.hpp"

namespace avdb {

AVDB_HD uint64_t zero_bytes_mask(uint64_t y) {  // bit 7 of each zero byte
  const uint64_t lo7 = 0x7F7F7F7F7F7F7F7Full;
  return ~(((y & lo7) + lo7) | y | lo7);
}

constexpr uint64_t kHiBits = 0x8080808080808080ull;

// Text pointers with an explicit address space, so byte reads compile to
// ds_read_u8 (LDS-staged window) or global_load_ubyte instead of flat loads.
typedef const __attribute__((address_space(3))) uint8_t* lds_cp;
typedef const __attribute__((address_space(3))) uint64_t* lds_cp64;
typedef const __attribute__((address_space(1))) uint8_t* glb_cp;

typedef const __attribute__((address_space(1))) uint64_t* glb_cp64;

// the 8-byte-word pointer of the same address space as a text pointer
template <class CP> struct Word64;
template <> struct Word64<lds_cp> { typedef lds_cp64 T; };
template <> struct Word64<glb_cp> { typedef glb_cp64 T; };
template <> struct Word64<const uint8_t*> { typedef const uint64_t* T; };  // host text (per-line entries)

// SWAR scan of s[0, n) eight bytes at a time (aligned words: an aligned word
// holding a byte of the text never leaves its LDS window / global page).  F maps a
// word to a mask with bit 7 set in every flagged byte; returns the index of the
// first flagged byte, or n.
template <class CP, class F>
AVDB_HD uint32_t swar_find(CP s, uint32_t n, F f) {
  if (n == 0) return 0;
  const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(s)) & 7u;
  const typename Word64<CP>::T w = reinterpret_cast<typename Word64<CP>::T>(s - mis);
  const uint32_t total = n + mis;
  uint64_t m = f(w[0]) & (~0ull << (8 * mis));
  uint32_t base = 0;
  while (!m) {
    base += 8;
    if (base >= total) return n;
    m = f(w[base >> 3]);
  }
  const uint32_t at = base + (uint32_t(__builtin_ctzll(m)) >> 3);
  return at >= total ? n : at - mis;
}

AVDB_HD uint64_t bytes_eq_mask(uint64_t x, uint8_t c) {
  return zero_bytes_mask(x ^ (0x0101010101010101ull * c));
}

// 8 bytes at aligned address a (bytes outside [lo,hi) read as 0x00)
__device__ __forceinline__ uint64_t text_word(uintptr_t a, const Heap& h) { return heap_word(a, h); }

// bit 7 set in every byte of x that is not an ASCII digit
AVDB_HD uint64_t nondigit_mask(uint64_t x) {
  const uint64_t d = x ^ 0x3030303030303030ull;
  return (((d & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | d) & kHiBits;
}

AVDB_HD bool is_ws(uint8_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}
AVDB_HD bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
AVDB_HD bool is_alnum(uint8_t c) {
  return is_digit(c) || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
}

// A workgroup's text window: the bytes of lines [base, last) staged in LDS as
// 16-byte words.  staged == false when it exceeds kStage (lanes then read the
// text from global memory).
constexpr uint32_t kStage = 36 * 1024;  // 4 workgroups per CU in 160 KB LDS

struct Window {
  uintptr_t a0;  // 16-aligned address of LDS byte 0
  bool staged;
};

// n16 16-byte words from a0 (16-aligned) into lds[0, n16), by kThreads threads,
// n16 <= kIter * kThreads: every thread issues all its loads before its first LDS
// store, so a workgroup's stage costs one memory round trip, not kIter (a load
// followed by its store in a loop waits vmcnt(0) every trip).  Words outside the
// text read as 0 (the bounded per-word path is taken only by a stage that reaches
// past either end of the text).
template <uint32_t kIter, uint32_t kThreads>
__device__ __forceinline__ void stage_copy(u32x4* lds, uintptr_t a0, uint32_t n16, const Heap& h) {
  const uint32_t tid = threadIdx.x;
  u32x4 v[kIter];
  if (a0 >= h.lo && a0 + 16 * uintptr_t(n16) <= h.hi) {
#pragma unroll
    for (uint32_t k = 0; k < kIter; ++k) {
      const uint32_t i = tid + k * kThreads;
      if (i < n16) v[k] = __builtin_nontemporal_load(gptr<u32x4>(a0 + 16 * uintptr_t(i)));
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kIter; ++k) {
      const uint32_t i = tid + k * kThreads;
      if (i < n16) {
        const uintptr_t a = a0 + 16 * uintptr_t(i);
        const uint64_t x = text_word(a, h), y = text_word(a + 8, h);
        v[k] = u32x4{uint32_t(x), uint32_t(x >> 32), uint32_t(y), uint32_t(y >> 32)};
      }
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < kIter; ++k) {
    const uint32_t i = tid + k * kThreads;
    if (i < n16) lds[i] = v[k];
  }
}

// kBatch false: the one-load-per-trip loop (fewer live registers while staging)
template <uint32_t kThreads, uint32_t kStageBytes = kStage, bool kBatch = true>
__device__ __forceinline__ Window stage_window(const Heap& h, size_t s0, size_t s1, u32x4* lds) {
  Window w;
  w.a0 = (h.lo + s0) & ~uintptr_t(15);
  const uintptr_t end = h.lo + s1;
  const size_t n16 = (end - w.a0 + 15) / 16;
  w.staged = n16 * 16 <= kStageBytes;
  if (w.staged) {
    if constexpr (kBatch) {
      stage_copy<(kStageBytes / 16 + kThreads - 1) / kThreads, kThreads>(lds, w.a0, uint32_t(n16), h);
    } else {
      for (size_t i = threadIdx.x; i < n16; i += kThreads) {
        const uintptr_t a = w.a0 + 16 * i;
        u32x4 v;
        if (a >= h.lo && a + 16 <= h.hi) {
          v = __builtin_nontemporal_load(gptr<u32x4>(a));
        } else {
          const uint64_t x = text_word(a, h), y = text_word(a + 8, h);
          v = u32x4{uint32_t(x), uint32_t(x >> 32), uint32_t(y), uint32_t(y >> 32)};
        }
        lds[i] = v;
      }
    }
  }
  __syncthreads();
  return w;
}

}  // namespace avdb
