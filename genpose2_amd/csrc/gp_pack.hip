// Host-side weight packing behind the C ABI (gp_weights_pack_host / gp_weights_pack / gp_weights_free):
// state-dict arrays -> the layouts the kernels stream, byte-identical to genpose2_amd/pack.py, so a host
// that is not Python (cgo, JNI, C++) can drive the library from a checkpoint's tensors.
//
// Replaces the reference's load path, PoseNet.load_ckpt -> net.load_state_dict
// (networks/posenet_agent.py:171-203), for the --dino none models: GFObjectPose score / energy
// (networks/posenet.py:27-124) and ScaleNet (networks/scalenet.py:12-31). Key names are the reference's
// model_state_dict keys.
//   * SA layers: Conv2d 1x1 + BatchNorm2d(eval) folded in float64, rounded once (pytorch_utils.py:58-106);
//     MFMA A-fragment order; layer 0's input channels permuted to [feats | xyz | pad] (pack.pack_encoder);
//     split-f16 hi/lo planes for every layer of levels 1-4 and layers 1-2 of level 0 (pack.pack_h16_fragments,
//     per-layer exponent).
//   * heads: first head layer split into its [pts 1024 | t 128 | pose 256] column blocks (scorenet.py:249),
//     fragments / transposes / split planes / activation bounds as pack.pack_heads.
//   * ScaleNet: plain copies.
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "gp_common.h"

namespace {

struct Tensor {
    const float* p;
    int64_t n;
};

struct StateDict {
    std::map<std::string, Tensor> m;
    std::string missing;
    const float* get(const std::string& k, int64_t numel) {
        auto it = m.find(k);
        if (it == m.end() || it->second.n != numel) {
            if (missing.empty())
                missing = k + (it == m.end() ? " (missing)" : " (size " + std::to_string(it->second.n) + ", want " +
                                                                  std::to_string(numel) + ")");
            return nullptr;
        }
        return it->second.p;
    }
};

// Light-config SA widths (arch.sa_branches): [level][branch] = {c_in + 3, h1, h2, h3 | 0}
const int kW[5][2][4] = {{{3, 16, 16, 32}, {3, 32, 32, 64}},
                         {{99, 64, 64, 128}, {99, 64, 96, 128}},
                         {{259, 128, 196, 256}, {259, 128, 196, 256}},
                         {{515, 256, 256, 512}, {515, 256, 384, 512}},
                         {{1027, 512, 512, 0}, {1027, 512, 512, 0}}};
constexpr double kBnEps = 1e-5;

int pad_to(int v, int a) { return (v + a - 1) / a * a; }

// (n_out, k_in) row-major -> A-fragment order packed[T][g][q][i][j] = W[16T + i][16g + 4q + j] (pack_a_fragments)
std::vector<float> pack_a(const std::vector<float>& w, int n_out, int k_in, int n_pad, int k_pad) {
    std::vector<float> out((size_t)n_pad * k_pad, 0.f);
    const int NT = n_pad / 16, KG = k_pad / 16;
    for (int T = 0; T < NT; ++T)
        for (int g = 0; g < KG; ++g)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < 16; ++i)
                    for (int j = 0; j < 4; ++j) {
                        const int r = 16 * T + i, c = 16 * g + 4 * q + j;
                        out[((((size_t)T * KG + g) * 4 + q) * 16 + i) * 4 + j] =
                            (r < n_out && c < k_in) ? w[(size_t)r * k_in + c] : 0.f;
                    }
    return out;
}

// e with max|w| * 2^e in [2^14, 2^15) (pack.split_exponent)
int split_exponent(const std::vector<float>& w) {
    float m = 0.f;
    for (float v : w) m = std::fmax(m, std::fabs(v));
    return m > 0.f ? 14 - (int)std::floor(std::log2((double)m)) : 0;
}

// bits of the f16 planes of x = w * 2^e in the v_mfma_f32_16x16x32_f16 A order (pack_h16_fragments):
// packed[T][c][plane][q][i][half][j4] = plane(W[16T + i][32c + 16 half + 4q + j4]); planes 2 (hi, lo) or
// 3 (hi, mid, lo: plane p = f16 of x minus the planes before it)
std::vector<uint32_t> pack_h16(const std::vector<float>& w, int n_out, int k_in, int e, int planes = 2) {
    const int NT = n_out / 16, KC = k_in / 32;
    std::vector<uint16_t> h((size_t)n_out * k_in * planes);
    const float s = std::ldexp(1.0f, e);
    for (int T = 0; T < NT; ++T)
        for (int c = 0; c < KC; ++c)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < 16; ++i)
                    for (int half = 0; half < 2; ++half)
                        for (int j4 = 0; j4 < 4; ++j4) {
                            float r = w[(size_t)(16 * T + i) * k_in + 32 * c + 16 * half + 4 * q + j4] * s;
                            for (int plane = 0; plane < planes; ++plane) {
                                const _Float16 v = (_Float16)r;
                                r = r - (float)v;
                                uint16_t bits;
                                std::memcpy(&bits, &v, 2);
                                h[((((((size_t)T * KC + c) * planes + plane) * 4 + q) * 16 + i) * 2 + half) * 4 + j4] = bits;
                            }
                        }
    std::vector<uint32_t> out(h.size() / 2);
    std::memcpy(out.data(), h.data(), h.size() * 2);
    return out;
}

// numpy's pairwise summation of n doubles (the inner loop of ndarray.sum along a contiguous axis)
double np_pairwise(const double* a, int64_t n) {
    if (n < 8) {
        double r = 0.0;   // numpy starts from -0.0 then adds; same result for our non-negative inputs
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

// max over rows of the row L1 norm in float64 (np.abs(w.astype(float64)).sum(1).max())
double max_row_l1(const float* w, int rows, int cols) {
    std::vector<double> r(cols);
    double m = 0.0;
    for (int o = 0; o < rows; ++o) {
        for (int c = 0; c < cols; ++c) r[c] = std::fabs((double)w[(size_t)o * cols + c]);
        m = std::fmax(m, np_pairwise(r.data(), cols));
    }
    return m;
}

struct Packer {
    std::vector<float> buf;
    size_t add(const float* p, size_t n) {   // appended at a 16-byte boundary; returns the float offset
        const size_t o = buf.size();
        buf.insert(buf.end(), p, p + n);
        buf.resize(buf.size() + (4 - buf.size() % 4) % 4, 0.f);
        return o;
    }
    size_t add(const std::vector<float>& v) { return add(v.data(), v.size()); }
    size_t add_bits(const std::vector<uint32_t>& v) {
        std::vector<float> f(v.size());
        std::memcpy(f.data(), v.data(), v.size() * 4);
        return add(f);
    }
};

// Conv2d 1x1 (no bias) + BatchNorm2d(eval) folded in float64 (weights.fold_conv_bn)
bool fold_conv_bn(StateDict& sd, const std::string& p, int n_out, int k_in, std::vector<float>& W, std::vector<float>& b) {
    const float* w = sd.get(p + ".conv.weight", (int64_t)n_out * k_in);
    const float* g = sd.get(p + ".bn.bn.weight", n_out);
    const float* be = sd.get(p + ".bn.bn.bias", n_out);
    const float* mu = sd.get(p + ".bn.bn.running_mean", n_out);
    const float* var = sd.get(p + ".bn.bn.running_var", n_out);
    if (!w || !g || !be || !mu || !var) return false;
    W.resize((size_t)n_out * k_in);
    b.resize(n_out);
    for (int o = 0; o < n_out; ++o) {
        const double sc = (double)g[o] / std::sqrt((double)var[o] + kBnEps);
        for (int c = 0; c < k_in; ++c) W[(size_t)o * k_in + c] = (float)((double)w[(size_t)o * k_in + c] * sc);
        b[o] = (float)((double)be[o] - (double)mu[o] * sc);
    }
    return true;
}

// pack.pack_encoder: the packed buffer (appended to P) and the [5][2][3][4] table relative to its start
bool pack_encoder(StateDict& sd, Packer& P, int64_t* table) {
    const size_t base = P.buf.size();
    for (int i = 0; i < 120; ++i) table[i] = -1;
    for (int lv = 0; lv < 5; ++lv) {
        const int c_prev = kW[lv][0][0] - 3;
        const int nl = lv < 4 ? 3 : 2;
        for (int br = 0; br < 2; ++br)
            for (int i = 0; i < nl; ++i) {
                const int n_out = kW[lv][br][i + 1], k_in = kW[lv][br][i];
                std::vector<float> W, b;
                const std::string p = "pts_encoder.SA_modules." + std::to_string(lv) + ".mlps." + std::to_string(br) +
                                      ".layer" + std::to_string(i);
                if (!fold_conv_bn(sd, p, n_out, k_in, W, b)) return false;
                int64_t* row = table + ((lv * 2 + br) * 3 + i) * 4;
                std::vector<float> packed;
                if (i == 0) {   // [xyz | feats] -> [feats | xyz | 0]
                    std::vector<float> wp((size_t)n_out * (c_prev + 16), 0.f);
                    for (int o = 0; o < n_out; ++o) {
                        for (int c = 0; c < c_prev; ++c) wp[(size_t)o * (c_prev + 16) + c] = W[(size_t)o * k_in + 3 + c];
                        for (int c = 0; c < 3; ++c) wp[(size_t)o * (c_prev + 16) + c_prev + c] = W[(size_t)o * k_in + c];
                    }
                    packed = pack_a(wp, n_out, c_prev + 16, pad_to(n_out, 16), c_prev + 16);
                } else {
                    packed = pack_a(W, n_out, k_in, pad_to(n_out, 16), pad_to(k_in, 16));
                }
                row[0] = (int64_t)(P.add(packed) - base);
                std::vector<float> bp(pad_to(n_out, 32), 0.f);
                std::copy(b.begin(), b.end(), bp.begin());
                row[1] = (int64_t)(P.add(bp) - base);
                if (lv >= 1 || i >= 1) {   // pack.enc_split_layer
                    const int np = pad_to(n_out, 32), kp = pad_to(k_in, 32);
                    std::vector<float> wq((size_t)np * kp, 0.f);
                    for (int o = 0; o < n_out; ++o) {
                        if (i == 0) {   // layer 0: [feats | xyz | 0]
                            for (int c = 0; c < c_prev; ++c) wq[(size_t)o * kp + c] = W[(size_t)o * k_in + 3 + c];
                            for (int c = 0; c < 3; ++c) wq[(size_t)o * kp + c_prev + c] = W[(size_t)o * k_in + c];
                        } else {
                            for (int c = 0; c < k_in; ++c) wq[(size_t)o * kp + c] = W[(size_t)o * k_in + c];
                        }
                    }
                    const int e = split_exponent(W);
                    row[2] = (int64_t)(P.add_bits(pack_h16(wq, np, kp, e)) - base);
                    row[3] = e;
                }
            }
    }
    return true;
}

// pack.pack_heads: field offsets (gp_head_weights order) in P
bool pack_heads(StateDict& sd, Packer& P, int64_t* f) {
    const std::string n = "pose_score_net.";
    const float* pe0_w = sd.get(n + "pose_encoder.0.weight", 256 * 9);
    const float* pe0_b = sd.get(n + "pose_encoder.0.bias", 256);
    const float* pe2_w = sd.get(n + "pose_encoder.2.weight", 256 * 256);
    const float* pe2_b = sd.get(n + "pose_encoder.2.bias", 256);
    const float* gfp = sd.get(n + "t_encoder.0.W", 64);
    const float* te_w = sd.get(n + "t_encoder.1.weight", 128 * 128);
    const float* te_b = sd.get(n + "t_encoder.1.bias", 128);
    const char* heads[3] = {"fusion_tail_rot_x", "fusion_tail_rot_y", "fusion_tail_trans"};
    const float *h1w[3], *h1b[3], *h2w[3], *h2b[3];
    for (int h = 0; h < 3; ++h) {
        h1w[h] = sd.get(n + heads[h] + ".0.weight", 256 * 1408);
        h1b[h] = sd.get(n + heads[h] + ".0.bias", 256);
        h2w[h] = sd.get(n + heads[h] + ".2.weight", 3 * 256);
        h2b[h] = sd.get(n + heads[h] + ".2.bias", 3);
        if (!h1w[h] || !h1b[h] || !h2w[h] || !h2b[h]) return false;
    }
    if (!pe0_w || !pe0_b || !pe2_w || !pe2_b || !gfp || !te_w || !te_b) return false;
    std::vector<float> w_pe0(pe0_w, pe0_w + 256 * 9), w_pe2(pe2_w, pe2_w + 256 * 256);
    std::vector<float> h1_pose((size_t)768 * 256), h1pts_t((size_t)1024 * 768), h1t_t((size_t)128 * 768), h1_b(768);
    std::vector<float> h2_w(9 * 256), h2_b(9), te_w_t(128 * 128);
    for (int h = 0; h < 3; ++h)
        for (int o = 0; o < 256; ++o) {
            const float* row = h1w[h] + (size_t)o * 1408;
            const int oo = h * 256 + o;
            for (int c = 0; c < 1024; ++c) h1pts_t[(size_t)c * 768 + oo] = row[c];
            for (int c = 0; c < 128; ++c) h1t_t[(size_t)c * 768 + oo] = row[1024 + c];
            for (int c = 0; c < 256; ++c) h1_pose[(size_t)oo * 256 + c] = row[1152 + c];
            h1_b[oo] = h1b[h][o];
        }
    for (int h = 0; h < 3; ++h) {
        for (int i = 0; i < 3 * 256; ++i) h2_w[h * 768 + i] = h2w[h][i];
        for (int i = 0; i < 3; ++i) h2_b[h * 3 + i] = h2b[h][i];
    }
    for (int r = 0; r < 128; ++r)
        for (int c = 0; c < 128; ++c) te_w_t[(size_t)c * 128 + r] = te_w[(size_t)r * 128 + c];
    f[0] = P.add(pack_a(w_pe0, 256, 9, 256, 16));
    f[1] = P.add(pe0_b, 256);
    f[2] = P.add(pack_a(w_pe2, 256, 256, 256, 256));
    f[3] = P.add(pe2_b, 256);
    f[4] = P.add(pack_a(h1_pose, 768, 256, 768, 256));
    f[5] = P.add(h2_w);
    f[6] = P.add(h2_b);
    f[7] = P.add(h1pts_t);
    f[8] = P.add(h1_b);
    f[9] = P.add(gfp, 64);
    f[10] = P.add(te_w_t);
    f[11] = P.add(te_b, 128);
    f[12] = P.add(h1t_t);
    const int e2 = split_exponent(w_pe2), eh = split_exponent(h1_pose);
    f[13] = P.add_bits(pack_h16(w_pe2, 256, 256, e2, 3));      // pack.HEAD_PLANES
    f[14] = P.add_bits(pack_h16(h1_pose, 768, 256, eh, 3));
    // split_constants: activation bounds, rounded to float32 then one step up
    float b0 = 0.f, b2 = 0.f;
    for (int i = 0; i < 256; ++i) {
        b0 = std::fmax(b0, std::fabs(pe0_b[i]));
        b2 = std::fmax(b2, std::fabs(pe2_b[i]));
    }
    const float v[4] = {(float)max_row_l1(pe0_w, 256, 9), b0, (float)max_row_l1(pe2_w, 256, 256), b2};
    float hsc[8];
    for (int i = 0; i < 4; ++i) hsc[i] = std::nextafter(v[i], INFINITY);
    hsc[4] = (float)e2;
    hsc[5] = (float)eh;
    hsc[6] = hsc[7] = 0.f;
    f[15] = P.add(hsc, 8);
    return true;
}

// pack.pack_scale: field offsets (gp_scale_weights order)
bool pack_scale(StateDict& sd, Packer& P, int64_t* f) {
    const char* keys[8] = {"axes_encoder.0.weight", "axes_encoder.0.bias", "axes_encoder.2.weight",
                           "axes_encoder.2.bias", "fusion_tail_length.0.weight", "fusion_tail_length.0.bias",
                           "fusion_tail_length.2.weight", "fusion_tail_length.2.bias"};
    const int64_t sz[8] = {256 * 180, 256, 256 * 256, 256, 256 * 1280, 256, 3 * 256, 3};
    for (int i = 0; i < 8; ++i) {
        const float* p = sd.get(keys[i], sz[i]);
        if (!p) return false;
        f[i] = P.add(p, sz[i]);
    }
    return true;
}

int pack_all(int kind, int n, const char* const* names, const float* const* data, const int64_t* numel, Packer& P,
             int64_t* fields, int64_t* enc_table) {
    GP_REQUIRE(kind >= GP_MODEL_SCORE && kind <= GP_MODEL_SCALE, "weights_pack: kind %d", kind);
    GP_REQUIRE(n >= 0 && (n == 0 || (names && data && numel)), "weights_pack: null arrays");
    StateDict sd;
    for (int i = 0; i < n; ++i) {
        GP_REQUIRE(names[i] && (data[i] || numel[i] == 0), "weights_pack: null entry %d", i);
        std::string k = names[i];
        if (k.rfind("module.", 0) == 0) k = k.substr(7);   // DataParallel prefix (weights.load_checkpoint)
        sd.m[k] = Tensor{data[i], numel[i]};
    }
    for (int i = 0; i < GP_PACK_NFIELDS; ++i) fields[i] = -1;
    bool ok;
    if (kind == GP_MODEL_SCALE) {
        ok = pack_scale(sd, P, fields + GP_PACK_SCALE);
    } else {
        fields[GP_PACK_ENC] = 0;
        ok = pack_encoder(sd, P, enc_table) && pack_heads(sd, P, fields + GP_PACK_HEADS);
    }
    if (!ok) {
        gp_set_error("weights_pack: state dict entry %s", sd.missing.c_str());
        return GP_ERR_INVALID;
    }
    return GP_OK;
}

}  // namespace

struct gp_weights {
    int kind;
    void* dev;
    size_t bytes;
    gp_head_weights heads;
    gp_scale_weights scale;
    int64_t table[120];
};

extern "C" int gp_weights_pack_host(int kind, int n, const char* const* names, const float* const* data,
                                    const int64_t* numel, float* out, size_t out_floats, size_t* need_floats,
                                    int64_t* fields, int64_t* enc_table) {
    GP_REQUIRE(need_floats && fields && enc_table, "weights_pack_host: null outputs");
    Packer P;
    const int rc = pack_all(kind, n, names, data, numel, P, fields, enc_table);
    if (rc) return rc;
    *need_floats = P.buf.size();
    if (out) {
        GP_REQUIRE(out_floats >= P.buf.size(), "weights_pack_host: out holds %zu floats, need %zu", out_floats,
                   P.buf.size());
        std::memcpy(out, P.buf.data(), P.buf.size() * sizeof(float));
    }
    return GP_OK;
}

extern "C" int gp_weights_pack(int kind, int n, const char* const* names, const float* const* data,
                               const int64_t* numel, gp_weights** out) {
    GP_REQUIRE(out, "weights_pack: null out");
    *out = nullptr;
    Packer P;
    int64_t fields[GP_PACK_NFIELDS];
    gp_weights* w = new gp_weights();
    int rc = pack_all(kind, n, names, data, numel, P, fields, w->table);
    if (rc) {
        delete w;
        return rc;
    }
    w->kind = kind;
    w->bytes = P.buf.size() * sizeof(float);
    if (hipMalloc(&w->dev, w->bytes) != hipSuccess ||
        hipMemcpy(w->dev, P.buf.data(), w->bytes, hipMemcpyHostToDevice) != hipSuccess) {
        if (w->dev) (void)hipFree(w->dev);
        delete w;
        return gp_check_launch("weights_pack: device upload");
    }
    const float* base = static_cast<const float*>(w->dev);
    auto at = [&](int64_t o) -> const float* { return o >= 0 ? base + o : nullptr; };
    if (kind == GP_MODEL_SCALE) {
        const float** s = reinterpret_cast<const float**>(&w->scale);
        for (int i = 0; i < 8; ++i) s[i] = at(fields[GP_PACK_SCALE + i]);
    } else {
        const float** h = reinterpret_cast<const float**>(&w->heads);
        for (int i = 0; i < 16; ++i) h[i] = at(fields[GP_PACK_HEADS + i]);
    }
    *out = w;
    return GP_OK;
}

extern "C" void gp_weights_free(gp_weights* w) {
    if (!w) return;
    if (w->dev) (void)hipFree(w->dev);
    delete w;
}

extern "C" const gp_head_weights* gp_weights_heads(const gp_weights* w) {
    return w && w->kind != GP_MODEL_SCALE ? &w->heads : nullptr;
}

extern "C" const gp_scale_weights* gp_weights_scale(const gp_weights* w) {
    return w && w->kind == GP_MODEL_SCALE ? &w->scale : nullptr;
}

extern "C" const float* gp_weights_encoder(const gp_weights* w, const int64_t** layer_off) {
    if (!w || w->kind == GP_MODEL_SCALE) return nullptr;
    if (layer_off) *layer_off = w->table;
    return static_cast<const float*>(w->dev);
}
