# A/B patch (round 5): the MEGA kernels (config E) test the boxes below a walked mega --
# its super group and the walked supers' cluster groups -- in the SCENE frame (pack_local_boxes' world boxes
# around the locally floored radii), with one margin per walked mega: the reference-rounding term from the
# mega's local distance bound pml = |o - S|_1 + Rg (the super group's record, S and Rg as lmask reads them),
# the slab-rounding term from the scene magnitudes pms = |o|_1 + w_cmax.  The per-lane frame rebuild
# (~12 VALU per box group, lmask) runs once per walked mega instead of once per group.  Margin proof:
# tests/box_cull_fuzz.c LOCAL = 2.
import sys
d = sys.argv[1]

def sub(path, old, new, count=1):
    p = f"{d}/{path}"; s = open(p).read()
    assert s.count(old) == count, (path, old[:80], s.count(old))
    s = s.replace(old, new); open(p, "w").write(s)

# ---- host: world cluster and super boxes, and their max |C|_1 + |H|_1
sub("rt_layout.hpp",
    "                             std::vector<float>& lgig, float& r2max, float& r2min, std::vector<float>* wmeg = nullptr) {",
    "                             std::vector<float>& lgig, float& r2max, float& r2min, std::vector<float>* wmeg = nullptr,\n"
    "                             std::vector<float>* wclo = nullptr, std::vector<float>* wsuo = nullptr, float* cmaxw = nullptr) {")
sub("rt_layout.hpp",
    "    if (wmeg) *wmeg = wme;\n",
    "    if (wmeg) *wmeg = wme;\n"
    "    // the world cluster and super boxes (the MEGA kernels' hybrid walk) and their largest |C|_1 + |H|_1\n"
    "    if (wclo) *wclo = wcl;\n"
    "    if (wsuo) *wsuo = wsu;\n"
    "    if (cmaxw) {\n"
    "        double cm = 0.0;\n"
    "        for (const std::vector<float>* v : {&wcl, &wsu})\n"
    "            for (size_t k = 0; k < 4 * (v->size() / kBoxFloats); ++k) {\n"
    "                float b[6];\n"
    "                get(*v, k, b);\n"
    "                if (!(b[3] > -INFINITY)) continue;\n"
    "                const double t = std::fabs((double)b[0]) + std::fabs((double)b[1]) + std::fabs((double)b[2]) + (double)b[3] +\n"
    "                                 (double)b[4] + (double)b[5];\n"
    "                if (std::isfinite(t)) cm = std::max(cm, t);\n"
    "            }\n"
    "        *cmaxw = up32(cm);\n"
    "    }\n")
# ---- context, upload, free, launch
sub("rt_kernel.hip",
    "    void* lbx64[4] = {}; void* lbx32[4] = {};       // local box levels: cluster boxes, supers, megas, gigas\n",
    "    void* lbx64[4] = {}; void* lbx32[4] = {};       // local box levels: cluster boxes, supers, megas, gigas\n"
    "    void* wbx64[2] = {}; void* wbx32[2] = {};       // world cluster and super boxes (the hybrid walk)\n"
    "    float w_cmax64 = 0, w_cmax32 = 0;\n")
sub("rt_kernel.hip",
    "        (void)hipFree(c->lbx64[lv]); (void)hipFree(c->lbx32[lv]);\n        c->lbx64[lv] = c->lbx32[lv] = nullptr;\n    }\n",
    "        (void)hipFree(c->lbx64[lv]); (void)hipFree(c->lbx32[lv]);\n        c->lbx64[lv] = c->lbx32[lv] = nullptr;\n    }\n"
    "    for (int lv = 0; lv < 2; ++lv) {\n        (void)hipFree(c->wbx64[lv]); (void)hipFree(c->wbx32[lv]);\n        c->wbx64[lv] = c->wbx32[lv] = nullptr;\n    }\n")
sub("rt_kernel.hip",
    "            pack_local_boxes(c64, L, q64, b64[0], b64[1], b64[2], b64[3], c->l_r2max64, c->l_r2min64);\n"
    "            std::vector<float> wme;\n"
    "            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme);\n",
    "            std::vector<float> w64[2], w32[2];\n"
    "            pack_local_boxes(c64, L, q64, b64[0], b64[1], b64[2], b64[3], c->l_r2max64, c->l_r2min64, nullptr, &w64[0],\n"
    "                             &w64[1], &c->w_cmax64);\n"
    "            std::vector<float> wme;\n"
    "            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme, &w32[0],\n"
    "                             &w32[1], &c->w_cmax32);\n"
    "            for (int lv = 0; lv < 2; ++lv) {\n"
    "                if ((rc = up(&c->wbx64[lv], w64[lv].data(), w64[lv].size() * sizeof(float))) != RT_OK) return rc;\n"
    "                if ((rc = up(&c->wbx32[lv], w32[lv].data(), w32[lv].size() * sizeof(float))) != RT_OK) return rc;\n"
    "            }\n")
sub("rt_kernel.hip",
    "    p.lgig = (const float*)(f64 ? c->lbx64[3] : c->lbx32[3]);\n",
    "    p.lgig = (const float*)(f64 ? c->lbx64[3] : c->lbx32[3]);\n"
    "    p.wclb = (const float*)(f64 ? c->wbx64[0] : c->wbx32[0]);\n"
    "    p.wsub = (const float*)(f64 ? c->wbx64[1] : c->wbx32[1]);\n"
    "    p.w_cmax = f64 ? c->w_cmax64 : c->w_cmax32;\n")
sub("rt_common.hpp",
    "    float l_r2max, l_hir2, l_isr;   // their margin constants: max local r2f, 48 u 0.5 / min, 8 u / sqrt(min)\n",
    "    float l_r2max, l_hir2, l_isr;   // their margin constants: max local r2f, 48 u 0.5 / min, 8 u / sqrt(min)\n"
    "    const float* wclb;         // the walk below a mega (hybrid): world cluster boxes (per super, 4) and world\n"
    "    const float* wsub;         //     super boxes (per mega, 4), BoxGroup layout\n"
    "    float w_cmax;              //     and their largest |C|_1 + |H|_1\n")
# ---- kernel
sub("rt_sweep.hpp",
    "        auto walk_super = [&](uint32_t sup) {\n",
    "        auto walk_super = [&](uint32_t sup, const f2& W3, const f2& W4) {\n")
sub("rt_sweep.hpp",
    "            if constexpr (MEGA) {\n                mask = lmask(load_lbox((cptr<float>)__builtin_assume_aligned(qa.lclb, 64), sup));\n            }\n",
    "            if constexpr (MEGA) {   // the hybrid walk: world cluster boxes, the walked mega's margin (W3, W4)\n"
    "                mask = box_mask(load_box((cptr<float>)__builtin_assume_aligned(qa.wclb, 32), sup), B0, B1, B2, W3, W4, btf());\n"
    "            }\n")
sub("rt_sweep.hpp",
    "                uint32_t smask = lmask(load_lbox(ls, nd));\n",
    "                // The boxes below mega nd in the scene frame (hybrid): the margin's reference-rounding term\n"
    "                // from the mega's local bound |o - S|_1 + Rg (its super group's record), the slab term from\n"
    "                // the scene magnitudes |o|_1 + w_cmax (tests/box_cull_fuzz.c LOCAL = 2)\n"
    "                const auto& qh = *cold_args<T>();\n"
    "                cptr<float> sr = ls + (32u * nd + 24u);\n"
    "                f2 ohxy;\n"
    "                float ohz;\n"
    "                if constexpr (sizeof(T) == 4) {\n"
    "                    ohxy = f2{o.x, o.y} - f2{sr[0], sr[1]};\n"
    "                    ohz = o.z - sr[2];\n"
    "                } else {\n"
    "                    ohxy = f2{(float)(o.x - (double)sr[0]), (float)(o.y - (double)sr[1])};\n"
    "                    ohz = (float)(o.z - (double)sr[2]);\n"
    "                }\n"
    "                const float pml = ((fabsf(ohxy.x) + fabsf(ohxy.y)) + fabsf(ohz)) + sr[3];\n"
    "                const float kw = __builtin_fmaf(__builtin_fmaf(pml, pml, qh.l_r2max), qh.l_hir2,\n"
    "                                                __builtin_fmaf(on + qh.w_cmax, qh.l_isr, 1.0f));\n"
    "                const f2 W3 = aixy * f2{kw, kw}, W4 = {aiz * kw, 0.0f};\n"
    "                uint32_t smask = box_mask(load_box((cptr<float>)__builtin_assume_aligned(qh.wsub, 32), nd), B0, B1, B2, W3,\n"
    "                                          W4, btf());\n")
sub("rt_sweep.hpp", "                    walk_super(sup);\n", "                    walk_super(sup, W3, W4);\n")
sub("rt_sweep.hpp", "                    walk_super(nd);\n", "                    walk_super(nd, B3, B4);\n")
