// fe_col.hpp -- one product-scanning column of the radix-2^32 multiply as ONE asm
// block: M v_mad_u64_u32 accumulate into acc (64-bit) with their carry-outs in M
// separate SGPR pairs, then M v_addc_co_u32 count the carries into top.  The carry of
// each MAC is read >= 2 instructions after it was written, so the 2 wait states gfx950
// needs between a VALU SGPR write and its read as carry-in come from the other
// instructions of the block instead of an s_nop per MAC (generated, see
// tools/microbench/femul.hip for the measurement).
#pragma once
#include <stdint.h>

template <int M> struct FeCol;

template <> struct FeCol<1> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, %2"
        : "+v"(acc), "+v"(top), "=&s"(c0)
        : "v"(x[0]), "v"(y[0])
        : "vcc");
  }
};

template <> struct FeCol<2> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1;
    asm("v_mad_u64_u32 %0, %2, %4, %6, %0\n\tv_mad_u64_u32 %0, %3, %5, %7, %0\n\ts_nop 0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\ts_nop 0\n\tv_addc_co_u32 %1, vcc, 0, %1, %3"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1)
        : "v"(x[0]), "v"(x[1]), "v"(y[0]), "v"(y[1])
        : "vcc");
  }
};

template <> struct FeCol<3> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2;
    asm("v_mad_u64_u32 %0, %2, %5, %8, %0\n\tv_mad_u64_u32 %0, %3, %6, %9, %0\n\tv_mad_u64_u32 %0, %4, %7, %10, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(y[0]), "v"(y[1]), "v"(y[2])
        : "vcc");
  }
};

template <> struct FeCol<4> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2, c3;
    asm("v_mad_u64_u32 %0, %2, %6, %10, %0\n\tv_mad_u64_u32 %0, %3, %7, %11, %0\n\tv_mad_u64_u32 %0, %4, %8, %12, %0\n\tv_mad_u64_u32 %0, %5, %9, %13, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, %5"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3])
        : "vcc");
  }
};

template <> struct FeCol<5> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2, c3, c4;
    asm("v_mad_u64_u32 %0, %2, %7, %12, %0\n\tv_mad_u64_u32 %0, %3, %8, %13, %0\n\tv_mad_u64_u32 %0, %4, %9, %14, %0\n\tv_mad_u64_u32 %0, %5, %10, %15, %0\n\tv_mad_u64_u32 %0, %6, %11, %16, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, %5\n\tv_addc_co_u32 %1, vcc, 0, %1, %6"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(c4)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4])
        : "vcc");
  }
};

template <> struct FeCol<6> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2, c3, c4, c5;
    asm("v_mad_u64_u32 %0, %2, %8, %14, %0\n\tv_mad_u64_u32 %0, %3, %9, %15, %0\n\tv_mad_u64_u32 %0, %4, %10, %16, %0\n\tv_mad_u64_u32 %0, %5, %11, %17, %0\n\tv_mad_u64_u32 %0, %6, %12, %18, %0\n\tv_mad_u64_u32 %0, %7, %13, %19, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, %5\n\tv_addc_co_u32 %1, vcc, 0, %1, %6\n\tv_addc_co_u32 %1, vcc, 0, %1, %7"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(c4), "=&s"(c5)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5])
        : "vcc");
  }
};

template <> struct FeCol<7> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2, c3, c4, c5, c6;
    asm("v_mad_u64_u32 %0, %2, %9, %16, %0\n\tv_mad_u64_u32 %0, %3, %10, %17, %0\n\tv_mad_u64_u32 %0, %4, %11, %18, %0\n\tv_mad_u64_u32 %0, %5, %12, %19, %0\n\tv_mad_u64_u32 %0, %6, %13, %20, %0\n\tv_mad_u64_u32 %0, %7, %14, %21, %0\n\tv_mad_u64_u32 %0, %8, %15, %22, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, %5\n\tv_addc_co_u32 %1, vcc, 0, %1, %6\n\tv_addc_co_u32 %1, vcc, 0, %1, %7\n\tv_addc_co_u32 %1, vcc, 0, %1, %8"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(c4), "=&s"(c5), "=&s"(c6)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]), "v"(y[6])
        : "vcc");
  }
};

template <> struct FeCol<8> {
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
    uint64_t c0, c1, c2, c3, c4, c5, c6, c7;
    asm("v_mad_u64_u32 %0, %2, %10, %18, %0\n\tv_mad_u64_u32 %0, %3, %11, %19, %0\n\tv_mad_u64_u32 %0, %4, %12, %20, %0\n\tv_mad_u64_u32 %0, %5, %13, %21, %0\n\tv_mad_u64_u32 %0, %6, %14, %22, %0\n\tv_mad_u64_u32 %0, %7, %15, %23, %0\n\tv_mad_u64_u32 %0, %8, %16, %24, %0\n\tv_mad_u64_u32 %0, %9, %17, %25, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, %3\n\tv_addc_co_u32 %1, vcc, 0, %1, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, %5\n\tv_addc_co_u32 %1, vcc, 0, %1, %6\n\tv_addc_co_u32 %1, vcc, 0, %1, %7\n\tv_addc_co_u32 %1, vcc, 0, %1, %8\n\tv_addc_co_u32 %1, vcc, 0, %1, %9"
        : "+v"(acc), "+v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(c4), "=&s"(c5), "=&s"(c6), "=&s"(c7)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]), "v"(y[6]), "v"(y[7])
        : "vcc");
  }
};
