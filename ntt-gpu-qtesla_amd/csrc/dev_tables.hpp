// dev_tables.hpp -- host-side construction and upload of the device twiddle
// tables of ntt_device.hpp, in the kernels' conventions:
//   forward (w, w') stored as (2^32 - w, w')          (ct_bfly)
//   inverse (w, w') stored centred as (ws, ws')        (sshoup_mul)
//   per-workgroup LDS images of the pass-2 lane twiddles + the bit-5 table
// Included by the translation unit that owns the __constant__ / __device__
// symbols (one per shared object).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ntt_device.hpp"
#include "ntt_large.hpp"
#include "ntt_big.hpp"
#include "ntt_eo.hpp"
#include "ntt_lat.hpp"
#include "params.hpp"

namespace qntt {

// (w, w') of twiddle index k of one direction, in the device convention
inline void dev_pair(const ParamSet &p, const Tables &t, bool inv, uint32_t k, uint32_t &w, uint32_t &wp)
{
    const std::vector<uint32_t> &tw = inv ? t.inv : t.fwd;
    if (inv) {
        const TwPair c = csigned_tw(tw[2 * k], p.q);
        w = c.x;
        wp = c.y;
    } else {
        w = 0u - tw[2 * k];
        wp = tw[2 * k + 1];
    }
}

// __constant__ table: n pairs, index k
inline std::vector<uint32_t> dev_const_table(const ParamSet &p, const Tables &t, bool inv)
{
    std::vector<uint32_t> v(2 * p.n);
    for (uint32_t k = 0; k < p.n; k++) dev_pair(p, t, inv, k, v[2 * k], v[2 * k + 1]);
    return v;
}

// LDS image (fill_tw2): entry e of stage bit b = tw2_b(e), lane t holds twiddle
// k = 2^(logn-1-b) + (Lp << (4-b)) + m with Lp = bitrev(lane) (see Lane);
// then the 32 bit-5 twiddles k = 32 + i.  `logn` is the geometry's (the
// 2048-point one for the large-n sub-trees) and kmap(k) the index in the
// direction's table (identity for n <= 2048).
template <class KMap>
inline std::vector<uint32_t> dev_tw2_image(const ParamSet &p, const Tables &t, bool inv, uint32_t logn, KMap kmap)
{
    std::vector<uint32_t> o(TW2_WORDS, 0);
    auto put = [&](int slot, uint32_t k) { dev_pair(p, t, inv, kmap(k), o[2 * slot], o[2 * slot + 1]); };
    const uint32_t lanes = logn == 11 ? 64 : 32;   // n = 1024: one entry column per 32-lane half (tw2_lanes)
    for (int e = 0; e < TW2_ENTRIES; e++) {
        const int b = e < 1 ? 4 : e < 3 ? 3 : e < 7 ? 2 : e < 15 ? 1 : 0;
        const uint32_t m = e - ((1u << (4 - b)) - 1);
        for (uint32_t lane = 0; lane < lanes; lane++) {
            const uint32_t Lp = logn == 11 ? bitrev(lane, 6) : bitrev(lane, 5);
            put(e * lanes + lane, (1u << (logn - 1 - b)) + (Lp << (4 - b)) + m);
        }
    }
    for (int i = 0; i < 32; i++) put(TW2_ENTRIES * 64 + i, 32u + i);
    return o;
}
inline std::vector<uint32_t> dev_tw2_image(const ParamSet &p, const Tables &t, bool inv)
{
    return dev_tw2_image(p, t, inv, p.logn, [](uint32_t k) { return k; });
}

// Large n = G * 2048: twiddle index k' of sub-tree B's 2048-point transform
// in the n-point table, k' = 2^s + m -> 2^s (G + B) + m (ntt_large.hpp)
inline uint32_t sub_tree_k(uint32_t kp, uint32_t G, uint32_t B)
{
    if (kp == 0) return 0;
    const uint32_t s = 31 - __builtin_clz(kp);
    return (kp - (1u << s)) + (1u << s) * (G + B);
}

// Tables of the large-n kernels of param set ps (3 or 4) to the current device
inline hipError_t upload_large_tables(int ps, const Tables &t)
{
    const ParamSet &p = *param_set(ps);
    const int idx = ps - LARGE_PS0;
    const uint32_t G = p.n / 2048;
    hipError_t e;
    for (int inv = 0; inv < 2; inv++) {
        uint2 sub[LARGE_GMAX][32] = {}, cross[4] = {}, b5[LARGE_GMAX][32] = {};
        for (uint32_t B = 0; B < G; B++) {
            for (uint32_t kp = 0; kp < 32; kp++)
                dev_pair(p, t, inv != 0, sub_tree_k(kp, G, B), sub[B][kp].x, sub[B][kp].y);
            const std::vector<uint32_t> img =
                dev_tw2_image(p, t, inv != 0, 11, [&](uint32_t kp) { return sub_tree_k(kp, G, B); });
            for (int i = 0; i < 32; i++) {   // the image's bit-5 pairs (c_bit5L)
                b5[B][i].x = img[TW2_BIT5_VEC4 * 4 + 2 * i];
                b5[B][i].y = img[TW2_BIT5_VEC4 * 4 + 2 * i + 1];
            }
            const size_t off = ((size_t)(idx * 2 + inv) * LARGE_GMAX + B) * TW2_VEC4 * 16;
            if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_tw2imgL), img.data(), TW2_WORDS * 4, off, hipMemcpyHostToDevice)) !=
                hipSuccess)
                return e;
        }
        for (uint32_t k = 1; k < G; k++) dev_pair(p, t, inv != 0, k, cross[k].x, cross[k].y);
        // sub-tree scale factors (c_fscale, ntt_large.hpp): c_{B,b} = T_B[k'] / T_0[k']
        // at k' = 2^(10-b) (the same ratio for every k' of stage b), and
        // F_B[j] = prod over the set bits b of j of c_{B,b}, as Shoup pairs
        {
            const std::vector<uint32_t> &tw = inv ? t.inv : t.fwd;
            auto mulq = [&](uint64_t a, uint64_t b) { return (uint32_t)(a * b % p.q); };
            auto powq = [&](uint64_t a, uint64_t e) {
                uint64_t r = 1;
                for (a %= p.q; e; e >>= 1, a = a * a % p.q)
                    if (e & 1) r = r * a % p.q;
                return (uint32_t)r;
            };
            uint2 fs[LARGE_GMAX][32] = {};
            for (uint32_t B = 0; B < G; B++) {
                uint32_t c[5];
                for (int b = 0; b < 5; b++) {
                    const uint32_t kp = 1u << (10 - b);
                    c[b] = mulq(tw[2 * sub_tree_k(kp, G, B)], powq(tw[2 * sub_tree_k(kp, G, 0)], p.q - 2));
                }
                for (uint32_t j = 0; j < 32; j++) {
                    uint32_t f = 1;
                    for (int b = 0; b < 5; b++)
                        if ((j >> b) & 1) f = mulq(f, c[b]);
                    fs[B][j].x = f;
                    fs[B][j].y = cshoup(f, p.q);
                }
            }
            if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_fscale), fs, sizeof fs, (size_t)(idx * 2 + inv) * sizeof fs,
                                       hipMemcpyHostToDevice)) != hipSuccess)
                return e;
        }
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_subtw), sub, sizeof sub, (size_t)(idx * 2 + inv) * sizeof sub,
                                   hipMemcpyHostToDevice)) != hipSuccess)
            return e;
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_cross), cross, sizeof cross, (size_t)(idx * 2 + inv) * sizeof cross,
                                   hipMemcpyHostToDevice)) != hipSuccess)
            return e;
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_bit5L), b5, sizeof b5, (size_t)(idx * 2 + inv) * sizeof b5,
                                   hipMemcpyHostToDevice)) != hipSuccess)
            return e;
    }
    uint2 last[3][LARGE_GMAX] = {};
    const uint32_t r32 = (uint32_t)((1ull << 32) % p.q);
    for (int rs = 0; rs < 3; rs++)
        for (uint32_t B = 0; B < G; B++) {   // n^-1 psi^-brv(G + B) (rs 1: times 2^32; rs 2: times 8 2^32,
                                              // the incomplete-domain product's (n/8)^-1), centred signed
            uint32_t w = (uint32_t)((uint64_t)t.n_inv * t.inv[2 * (G + B)] % p.q);
            if (rs) w = (uint32_t)((uint64_t)w * r32 % p.q);
            if (rs == 2) w = (uint32_t)((uint64_t)w * 8 % p.q);
            const TwPair c = csigned_tw(w, p.q);
            last[rs][B].x = c.x;
            last[rs][B].y = c.y;
        }
    return hipMemcpyToSymbol(HIP_SYMBOL(c_lastinv), last, sizeof last, (size_t)idx * sizeof last, hipMemcpyHostToDevice);
}

// Tables of the wave-per-polynomial n = 4096 / 8192 transforms (ntt_big.hpp):
// the uniform pass-1 twiddles k < R and the LDS image (lane table of every
// chunk, then the bit-5 table), tests/test_big_dataflow.py::lane_k
inline hipError_t upload_big_tables(int ps, const Tables &t)
{
    const ParamSet &p = *param_set(ps);
    const int idx = ps - LARGE_PS0;
    const uint32_t L = p.logn, R = 1u << (L - 6), NC = L - 11, CH = 1u << NC;
    hipError_t e;
    for (int inv = 0; inv < 2; inv++) {
        uint2 tw[BIG_RMAX] = {};
        for (uint32_t k = 0; k < R; k++) dev_pair(p, t, inv != 0, k, tw[k].x, tw[k].y);
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_bigtw), tw, sizeof tw, (size_t)(idx * 2 + inv) * sizeof tw,
                                   hipMemcpyHostToDevice)) != hipSuccess)
            return e;
        const uint32_t lane_pairs = TW2_ENTRIES * 64 * CH;
        std::vector<uint32_t> o(2 * (lane_pairs + R), 0);
        auto put = [&](uint32_t slot, uint32_t k) { dev_pair(p, t, inv != 0, k, o[2 * slot], o[2 * slot + 1]); };
        for (uint32_t c = 0; c < CH; c++)
            for (int ent = 0; ent < TW2_ENTRIES; ent++) {
                const int b = ent < 1 ? 4 : ent < 3 ? 3 : ent < 7 ? 2 : ent < 15 ? 1 : 0;
                const uint32_t m = ent - ((1u << (4 - b)) - 1);
                for (uint32_t lane = 0; lane < 64; lane++)
                    put((c * TW2_ENTRIES + ent) * 64 + lane,
                        (1u << (L - 1 - b)) + ((c + (bitrev(lane, 6) << NC)) << (4 - b)) + m);
            }
        for (uint32_t i = 0; i < R; i++) put(lane_pairs + i, R + i);   // bit-5 stage: k = 2^M + m + H h
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_bigimg), o.data(), o.size() * 4,
                                   (size_t)(idx * 2 + inv) * BIG_IMG_VEC4_MAX * 16, hipMemcpyHostToDevice)) != hipSuccess)
            return e;
    }
    return hipSuccess;
}

// Upload every table of the parameter sets to the current device.
inline hipError_t upload_device_tables(const Tables *tabs /* [NPARAM_SETS] */)
{
    const void *syms[3][2] = {{HIP_SYMBOL(c_fwd0), HIP_SYMBOL(c_inv0)},
                              {HIP_SYMBOL(c_fwd1), HIP_SYMBOL(c_inv1)},
                              {HIP_SYMBOL(c_fwd2), HIP_SYMBOL(c_inv2)}};
    for (int ps = 0; ps < 3; ps++)
        for (int inv = 0; inv < 2; inv++) {
            const ParamSet &p = *param_set(ps);
            const std::vector<uint32_t> c = dev_const_table(p, tabs[ps], inv != 0);
            hipError_t e = hipMemcpyToSymbol(syms[ps][inv], c.data(), c.size() * 4, 0, hipMemcpyHostToDevice);
            if (e != hipSuccess) return e;
            const std::vector<uint32_t> img = dev_tw2_image(p, tabs[ps], inv != 0);
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_tw2img), img.data(), TW2_WORDS * 4,
                                  (size_t)(ps * 2 + inv) * TW2_WORDS * 4, hipMemcpyHostToDevice);
            if (e != hipSuccess) return e;
        }
    for (int ps = LARGE_PS0; ps < LARGE_PS0 + LARGE_NPS; ps++) {
        hipError_t e = upload_large_tables(ps, tabs[ps]);
        if (e != hipSuccess) return e;
        if ((e = upload_big_tables(ps, tabs[ps])) != hipSuccess) return e;
#ifdef NTT_EO
        if (ps == LARGE_PS0 + 1) {
            // n = 8192 even/odd combine (ntt_eo.hpp): w_k = psi^(2k+1), CT index 4096 + brv12(k)
            std::vector<uint32_t> c(2 * 2 * 4096);
            for (int inv = 0; inv < 2; inv++)
                for (uint32_t k = 0; k < 4096; k++)
                    dev_pair(*param_set(ps), tabs[ps], inv != 0, 4096u + bitrev(k, 12), c[(inv * 4096 + k) * 2],
                             c[(inv * 4096 + k) * 2 + 1]);
            if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_eotw), c.data(), c.size() * 4, 0, hipMemcpyHostToDevice)) != hipSuccess)
                return e;
            // the split form: lambda_l = psi^(+-2 l) (Shoup pairs), mu = psi^(+-(2 k0 + 1)),
            // k0 = 128 brv5(I) + 64 c + 128 par (ntt_eo.hpp, EO_TWJIT)
            const ParamSet &p8 = *param_set(ps);
            const Tables &t8 = tabs[ps];
            uint2 lam[2][64], mu[2][2][2][16];
            for (int inv = 0; inv < 2; inv++) {
                const uint32_t g = inv ? t8.inv[2 * 4096] : t8.fwd[2 * 4096];   // psi^(+-1)
                const uint32_t g2 = (uint32_t)((uint64_t)g * g % p8.q);
                uint64_t x = 1;
                for (uint32_t l = 0; l < 64; l++, x = x * g2 % p8.q) {
                    lam[inv][l].x = (uint32_t)x;
                    lam[inv][l].y = shoup((uint32_t)x, p8.q);
                }
                for (uint32_t par = 0; par < 2; par++)
                    for (uint32_t cc = 0; cc < 2; cc++)
                        for (uint32_t i = 0; i < 16; i++) {
                            const uint32_t k0 = 128u * bitrev(i, 5) + 64u * cc + 128u * par;
                            dev_pair(p8, t8, inv != 0, 4096u + bitrev(k0, 12), mu[inv][par][cc][i].x, mu[inv][par][cc][i].y);
                        }
            }
            if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_eolam), lam, sizeof lam, 0, hipMemcpyHostToDevice)) != hipSuccess) return e;
            if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_eomu), mu, sizeof mu, 0, hipMemcpyHostToDevice)) != hipSuccess) return e;
        }
#endif
        // full n-point tables of the latency kernels (ntt_lat.hpp)
        for (int inv = 0; inv < 2; inv++) {
            const std::vector<uint32_t> c = dev_const_table(*param_set(ps), tabs[ps], inv != 0);
            e = ps == LARGE_PS0 ? hipMemcpyToSymbol(HIP_SYMBOL(g_lattw3), c.data(), c.size() * 4, (size_t)inv * c.size() * 4,
                                                    hipMemcpyHostToDevice)
                                : hipMemcpyToSymbol(HIP_SYMBOL(g_lattw4), c.data(), c.size() * 4, (size_t)inv * c.size() * 4,
                                                    hipMemcpyHostToDevice);
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

}  // namespace qntt
