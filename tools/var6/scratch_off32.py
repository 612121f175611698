"""A/B patch (round 6): PScratch record addresses as one 32-bit offset from the wave's scratch base (an SGPR pair), so
a record access is global_{load,store} voffset, saddr instead of 64-bit VGPR pointer arithmetic (v_mul_lo_u32 for the
slot offset, two v_lshl_add_u64): the slot's region offset as a 24-bit multiply of sbytes / 256 (sbytes is a multiple
of 256 and below 2^32; slot < 8), every per-wave offset below 2^32 (the scratch of one wave is < 200 MB at spp 2^20).
Bit-identical results (addressing only)."""
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"
s = open(p).read()
rep = [
('''    __device__ __forceinline__ uint32_t map(uint32_t q) const {
        if (wide & 2u) return *(const uint32_t*)(base + 4u * q);
        return from16(*(const uint16_t*)(base + 2u * q));
    }''', '''    // slot s's record region: vbytes + s * sbytes as one 24-bit multiply (sbytes % 256 == 0, s < 8), so every record
    // address is the wave's base (SGPRs) plus a 32-bit lane offset (global_* voffset, saddr)
    __device__ __forceinline__ uint32_t soff(uint32_t s) const { return vbytes + (__umul24(s, sbytes >> 8) << 8); }
    __device__ __forceinline__ uint32_t map(uint32_t q) const {
        if (wide & 2u) return *(const uint32_t*)(base + 4u * q);
        return from16(*(const uint16_t*)(base + 2u * q));
    }'''),
('''    __device__ __forceinline__ T& y(uint32_t s, uint32_t i) const {
        return *(T*)(base + vbytes + s * sbytes + i * (uint32_t)sizeof(T));
    }
    __device__ __forceinline__ C3<T>& c(uint32_t s, uint32_t i) const {
        return *(C3<T>*)(base + vbytes + s * sbytes + (P + 3u * i) * (uint32_t)sizeof(T));
    }''', '''    __device__ __forceinline__ T& y(uint32_t s, uint32_t i) const {
        return *(T*)(base + (soff(s) + i * (uint32_t)sizeof(T)));
    }
    __device__ __forceinline__ C3<T>& c(uint32_t s, uint32_t i) const {
        return *(C3<T>*)(base + (soff(s) + (P + 3u * i) * (uint32_t)sizeof(T)));
    }'''),
('''    __device__ __forceinline__ uint32_t e(uint32_t s, uint32_t i) const {
        const char* b = base + vbytes + s * sbytes + 4u * P * (uint32_t)sizeof(T);
        return (wide & 1u) ? *(const uint32_t*)(b + 4u * i) : (uint32_t) * (const uint8_t*)(b + i);
    }
    __device__ __forceinline__ void set_e(uint32_t s, uint32_t i, uint32_t v) const {
        char* b = base + vbytes + s * sbytes + 4u * P * (uint32_t)sizeof(T);
        if (wide & 1u) *(uint32_t*)(b + 4u * i) = v;
        else *(uint8_t*)(b + i) = (uint8_t)v;
    }''', '''    __device__ __forceinline__ uint32_t e(uint32_t s, uint32_t i) const {
        const uint32_t o = soff(s) + 4u * P * (uint32_t)sizeof(T);
        return (wide & 1u) ? *(const uint32_t*)(base + (o + 4u * i)) : (uint32_t) * (const uint8_t*)(base + (o + i));
    }
    __device__ __forceinline__ void set_e(uint32_t s, uint32_t i, uint32_t v) const {
        const uint32_t o = soff(s) + 4u * P * (uint32_t)sizeof(T);
        if (wide & 1u) *(uint32_t*)(base + (o + 4u * i)) = v;
        else *(uint8_t*)(base + (o + i)) = (uint8_t)v;
    }'''),
]
for a, b in rep:
    assert a in s, a[:60]
    s = s.replace(a, b)
open(p, "w").write(s)
