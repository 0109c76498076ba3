// phd_palette.cpp -- the palette's decision logic, run on the host between the
// two device passes (K1 histogram -> decisions -> Kcut/K3 sums).
//
// It reproduces, on the TL-sized group histogram alone, what the reference's
// get_color_palette does with its per-pixel linked lists
// (src/color_quantization.c:652-684):
//  * find_valid_octree_parents (:174-203): stable insertion sort
//    (custom_sort, src/utilities.c:132-153) by the float32 saliency
//    (:588-595) through compare_quantities (:601-611), whose `(int)` of the
//    float difference is x86 cvttss2si -> INT_MIN for |d| >= 2^31 or NaN;
//  * group_irregular_pixels (:342-479) as per-group keep rules: a group with one
//    nearest parent is spliced whole; a tie sends every pixel to the FIRST tied
//    parent (get_distance_pixel_to_parent has no return statement; at -O0 it
//    returns the pixel pointer's bits, identical for all candidates), appended
//    through the parent's stale tail pointer: the pixels that fit the tail node
//    survive, and on overflow only the group's last pixel survives as a
//    dangling node until the next event on that parent replaces it.
#include <algorithm>
#include <cmath>
#include <climits>
#include <cstring>

#include "phd_host.h"

namespace phd {

bool validate_config(const phd_config& c, std::string* why) {
    auto fail = [&](const char* m) { *why = m; return false; };
    if (c.h_partitions <= 0 || c.s_partitions <= 0 || c.v_partitions <= 0)
        return fail("h/s/v_partitions must be positive (initialize_octree, color_quantization.c:28)");
    if (360 % c.h_partitions != 0)
        return fail("h_partitions must divide 360: otherwise arm_octree indexes past the hue grid "
                    "(color_quantization.c:41,143; undefined behaviour in the reference)");
    if (!(c.black_thresh >= 0 && c.black_thresh < 1) || !(c.gray_thresh >= 0 && c.gray_thresh < 1))
        return fail("black_thresh and gray_thresh must lie in [0, 1)");
    if (!(c.coverage_thresh <= 1.0))
        return fail("coverage_thresh must be <= 1 (find_valid_octree_parents never terminates "
                    "otherwise, color_quantization.c:202)");
    if (c.linked_list_size <= 0) return fail("linked_list_size must be positive");
    if (c.radius_partitions <= 0 || c.angle_partitions <= 0)
        return fail("radius/angle_partitions must be positive");
    if ((long)c.radius_partitions * c.angle_partitions > 65535)
        return fail("radius_partitions * angle_partitions must be <= 65535");
    if (c.blur_cutoff_ratio_denom <= 0) return fail("blur_cutoff_ratio_denom must be positive");
    long tl = (long)c.h_partitions * c.s_partitions * c.v_partitions + c.v_partitions + 1;
    if (tl > 4096) return fail("h*s*v + v + 1 must be <= 4096 groups");
    if (c.s_partitions > 127) return fail("s_partitions must be <= 127 (int8 saturation-class table)");
    return true;
}

GridParams make_grid(const phd_config& c) {
    GridParams g{};
    g.hp = c.h_partitions;
    g.sp = c.s_partitions;
    g.vp = c.v_partitions;
    g.ng = c.v_partitions;                              // num_grays = v_parts, :27
    g.tl = g.hp * g.sp * g.vp + g.ng + 1;
    g.Lh = 360 / g.hp;                                  // integer division, :41
    g.Ls = (1 - c.gray_thresh) / g.sp;
    g.Lv = (1 - c.black_thresh) / g.vp;
    g.bt = c.black_thresh;
    g.gt = c.gray_thresh;
    return g;
}

GroupCenters make_centers(const GridParams& g) {
    GroupCenters gc;
    gc.h.assign(g.tl, 0.0);
    gc.s.assign(g.tl, 0.0);
    gc.v.assign(g.tl, 0.0);
    const double half_h = g.Lh / 2, s_offs = g.Ls / 2 + g.gt, v_offs = g.Lv / 2 + g.bt;
    for (int h = 0; h < g.hp; h++)
        for (int s = 0; s < g.sp; s++)
            for (int v = 0; v < g.vp; v++) {
                const int i = h * g.sp * g.vp + s * g.vp + v;
                gc.h[i] = h * g.Lh + half_h;
                gc.s[i] = s * g.Ls + s_offs;
                gc.v[i] = v * g.Lv + v_offs;
            }
    const double l_gray = (1.0f - g.bt) / (double)g.ng;  // :78 (1.0f promotes exactly)
    for (int j = 0; j < g.ng; j++) gc.v[g.hp * g.sp * g.vp + j] = l_gray * j + v_offs;
    return gc;                                            // black group stays (0, 0, 0)
}

void make_class_tables(const GridParams& g, FastCls* fc, ClassTables* t) {
    // every entry is the reference's own double expression (rgb2hsv,
    // src/image_processing.c:388-414; arm_octree, src/color_quantization.c:131-145)
    memset(t, 0, sizeof(*t));
    for (int k = 0; k < 256; k++) {
        const double v = (k == 255) ? 0.999999 : (double)k / 255.0;
        ClsEnt& e = t->ent[k];
        int vcol = -1, vgray = 0;
        if (v >= g.bt) {
            vcol = (int)((v - g.bt) / g.Lv);
            vgray = (int)((double)((int)(v - g.bt) * g.ng) / (1 - g.bt));
        }
        const int gray_id = g.tl - (g.ng + 1) + vgray;
        e.vpack = (int)(((unsigned)gray_id << 16) | ((unsigned)vcol & 0xFFFFu));
        // Si for every min <= max: s = max == 0 ? 0 : (d == max ? 0.999999 : d / max)
        const double mx = (double)k / 255.0;
        for (int kd = 0; kd <= k; kd++) {
            const double mn = (double)(k - kd) / 255.0, d = mx - mn;
            const double s = mx == 0 ? 0.0 : (d == mx ? 0.999999 : d / mx);
            t->si8[k * 256 + kd] = (signed char)(s < g.gt ? -1 : (int)((s - g.gt) / g.Ls));
        }
    }
    fc->lh = 360 / g.hp;
    // threshold form of si8 (ClsEnt::thr); valid while Si is non-decreasing
    // in kd and takes at most kSiThresholds non-negative values
    bool mono = g.sp <= kSiThresholds;
    for (int k = 0; k < 256 && mono; k++) {
        unsigned short thr[kSiThresholds];
        for (int j = 0; j < kSiThresholds; j++) thr[j] = 0xFFFF;
        for (int kd = 0; kd <= k; kd++) {
            const int si = t->si8[k * 256 + kd];
            if (kd > 0 && si < t->si8[k * 256 + kd - 1]) mono = false;
            for (int j = 0; j <= si && j < kSiThresholds; j++)
                if (thr[j] == 0xFFFF) thr[j] = (unsigned short)kd;
        }
        for (int i = 0; i < kSiThresholds / 2; i++)
            t->ent[k].thr[i] = (unsigned)thr[2 * i] | ((unsigned)thr[2 * i + 1] << 16);
    }
    fc->use_thr = mono ? 1 : 0;
    // K1 table (k1.hip): a code per (kmax, kd <= kmax): 0 .. sp*vp-1 colour
    // (Si * vp + Vi), sp*vp + (group - gray_start) for the gray / black groups
    const int gs = g.tl - g.ng - 1, sv = g.sp * g.vp;
    t->codes_ok = sv + g.ng + 1 <= 256 && g.tl <= 4095;
    for (int k = 0; k < 256 && t->codes_ok; k++) {
        const int vcol = (int)(short)(t->ent[k].vpack & 0xFFFF), gray_id = (int)((unsigned)t->ent[k].vpack >> 16);
        for (int kd = 0; kd <= k; kd++) {
            const int si = t->si8[k * 256 + kd];
            int code;
            if (vcol < 0) code = sv + (g.tl - 1 - gs);              // black (v < bt)
            else if (si < 0) code = sv + (gray_id - gs);            // gray (s < gt)
            else code = si * g.vp + vcol;
            if (code < 0 || code > 255) t->codes_ok = 0;
            t->code8[k * 256 + kd] = (unsigned char)code;
            t->code_tri[k * (k + 1) / 2 + kd] = (unsigned char)code;
        }
    }
    t->inv[0] = 0.0;
    for (int k = 1; k < 256; k++) t->inv[k] = 1.0 / (double)k;
    fc->k1t_cshift = k1t_cshift(g, *t);
    fc->k1t_cshift2 = fc->k1t_cshift >= 0 ? k1t_cshift2(g, *t) : -1;
}

namespace {

float saliency(unsigned q, double s, double v, float qw, float svw) {
    const float s_v = (float)(s * v);
    const float sal = (float)(int)q * (qw + svw * s_v);
    return sal * 1000;
}

double node_distance(const GridParams& g, const GroupCenters& c, int gi, int pi) {
    const int gray_start = g.tl - (g.ng + 1), black = g.tl - 1;
    if (gi < gray_start && pi < gray_start) {
        double hd = std::fabs(c.h[gi] - c.h[pi]);
        if (hd > 180) hd = 360 - hd;
        hd *= (1.0) / (360.0);
        const double sd = c.s[gi] - c.s[pi], vd = c.v[gi] - c.v[pi];
        return hd * hd + sd * sd + vd * vd;
    }
    const bool gray_i = gray_start <= gi && gi < black, gray_p = gray_start <= pi && pi < black;
    if ((gray_i && pi < gray_start) || (gray_p && gi < gray_start)) {
        const double sd = c.s[gi] - c.s[pi], vd = c.v[gi] - c.v[pi];
        return sd * sd + vd * vd;
    }
    const double vd = c.v[gi] - c.v[pi];
    return vd * vd;
}

// compare_quantities(x, y) < 0 for the element x being inserted and its left
// neighbour y, i.e. (int)(y - x) < 0 as the x86 conversion behaves (INT_MIN
// for |d| >= 2^31 or NaN): the insertion sort moves x past y.
inline bool moves_past(float y, float x) {
    const float d = y - x;
    return !(d > -1.0f && d < 2147483648.0f);
}

}  // namespace

std::vector<uint16_t> make_near_order(const GridParams& g, const GroupCenters& gc) {
    const int tl = g.tl;
    std::vector<uint16_t> near;
    if (tl > kNearMaxGroups) return near;
    near.resize((size_t)tl * tl);
    std::vector<double> d(tl);
    for (int i = 0; i < tl; i++) {
        for (int p = 0; p < tl; p++) d[p] = node_distance(g, gc, i, p);
        uint16_t* row = near.data() + (size_t)i * tl;
        for (int p = 0; p < tl; p++) row[p] = (uint16_t)p;
        std::sort(row, row + tl, [&](uint16_t a, uint16_t b) { return d[a] < d[b] || (d[a] == d[b] && a < b); });
    }
    return near;
}

bool decide_palette(const GridParams& g, const GroupCenters& gc, const unsigned* hist, long n_hsv,
                    const phd_config& cfg, PaletteDecision* out, const uint16_t* near) {
    const int tl = g.tl;
    const int L = cfg.linked_list_size;
    // ---- ordering by saliency: custom_sort's insertion sort (swap while
    // compare < 0).  x moves left past its neighbours while moves_past holds,
    // so its place is the first neighbour, scanning left, where it fails.  The
    // sorted prefix is a list of blocks (<= 2 kBlk entries, saliency max/min
    // each): a block whose max or min alone shows that x moves past all of it
    // (fl(y - x) is monotone in y) is skipped whole, one block is scanned, and
    // an insertion shifts one block, so nothing is O(tl^2) in memory traffic.
    std::vector<float> sal(tl);
    for (int i = 0; i < tl; i++)
        sal[i] = saliency(hist[i], gc.s[i], gc.v[i], cfg.quantity_weight, cfg.saturation_value_weight);
    constexpr int kBlk = 16;
    struct Blk {
        int n = 0;
        float mx = 0, mn = 0;
        int id[2 * kBlk + 1];
        float sv[2 * kBlk + 1];
        void bounds() {
            mx = mn = sv[0];
            for (int t = 1; t < n; t++) mx = std::max(mx, sv[t]), mn = std::min(mn, sv[t]);
        }
    };
    std::vector<Blk> pool(1);
    pool.reserve(tl / kBlk + 2);
    std::vector<int> blocks{0};                          // block order
    for (int i = 0; i < tl; i++) {
        const float x = sal[i];
        int b = (int)blocks.size() - 1, pos = 0;         // insert at (blocks[b], pos)
        for (; b >= 0; b--) {
            const Blk& k = pool[blocks[b]];
            // max <= x - 1: every y <= max moves; min >= x + 2^31: every y >= min moves
            if (k.n == 0 || !(k.mx - x > -1.0f) || !(k.mn - x < 2147483648.0f)) continue;
            int p = k.n;
            while (p > 0 && moves_past(k.sv[p - 1], x)) p--;
            if (p > 0) {
                pos = p;
                break;
            }
        }
        if (b < 0) b = 0, pos = 0;                       // x goes to the front
        Blk& k = pool[blocks[b]];
        std::memmove(&k.id[pos + 1], &k.id[pos], sizeof(int) * (k.n - pos));
        std::memmove(&k.sv[pos + 1], &k.sv[pos], sizeof(float) * (k.n - pos));
        k.id[pos] = i;
        k.sv[pos] = x;
        if (k.n++ == 0) k.mx = k.mn = x;
        else k.mx = std::max(k.mx, x), k.mn = std::min(k.mn, x);
        if (k.n > 2 * kBlk) {                             // split: the upper half to a new block
            pool.emplace_back();
            Blk& a = pool[blocks[b]];
            Blk& c2 = pool.back();
            c2.n = a.n - kBlk;
            std::memcpy(c2.id, a.id + kBlk, sizeof(int) * c2.n);
            std::memcpy(c2.sv, a.sv + kBlk, sizeof(float) * c2.n);
            a.n = kBlk;
            a.bounds();
            c2.bounds();
            blocks.insert(blocks.begin() + b + 1, (int)pool.size() - 1);
        }
    }
    std::vector<int> order;
    order.reserve(tl);
    for (int b : blocks) order.insert(order.end(), pool[b].id, pool[b].id + pool[b].n);
    int goal = (int)((double)n_hsv * cfg.coverage_thresh);
    int np = -1;
    for (int i = 0; i < tl; i++) {
        goal -= (int)hist[order[i]];
        if (goal <= 0) {
            np = i + 1;
            break;
        }
    }
    if (np < 0) {
        set_error("find_valid_octree_parents: coverage goal not reachable");
        return false;
    }
    out->parents.assign(order.begin(), order.begin() + np);
    out->rules.assign(tl, GroupRule{-1, 0, 0, 0, 0xFFFFFFFFu, 0u});
    out->kept.assign(np, 0);
    out->off.assign(np, 0.0);
    out->search.clear();

    std::vector<int> tail_fill(np), dangling(np, -1);
    std::vector<char> is_parent(tl, 0);
    for (int k = 0; k < np; k++) {
        const int p = out->parents[k];
        is_parent[p] = 1;
        const long q = hist[p];
        tail_fill[k] = q == 0 ? 0 : (int)((q - 1) % L) + 1;
        out->rules[p].slot = k;
        out->kept[k] = q;
        out->off[k] = 180 - gc.h[p];
    }
    std::vector<double> dist(np);
    std::vector<int> slot_of(tl, -1);
    for (int k = 0; k < np; k++) slot_of[out->parents[k]] = k;
    for (int i = 0; i < tl; i++) {
        if (hist[i] == 0 || is_parent[i]) continue;
        double best = (double)tl * tl;                    // :368
        int nmin = 0, k = 0;
        if (near) {
            // the nearest parents are the first parents of i's distance order;
            // ties are adjacent there: count them, keep the first in palette order
            const uint16_t* row = near + (size_t)i * tl;
            int a = 0;
            while (slot_of[row[a]] < 0) a++;
            best = node_distance(g, gc, i, row[a]);
            k = slot_of[row[a]];
            nmin = 1;
            for (a++; a < tl; a++) {
                const int p = row[a];
                if (slot_of[p] < 0) continue;
                if (node_distance(g, gc, i, p) != best) break;
                nmin++;
                k = std::min(k, slot_of[p]);
            }
        } else {
            for (int kk = 0; kk < np; kk++) {
                const double d = node_distance(g, gc, i, out->parents[kk]);
                if (d < best) {
                    best = d;
                    nmin = 1;
                } else if (d == best) {
                    nmin++;
                }
                dist[kk] = d;
            }
            while (dist[k] != best) k++;                  // first nearest, valid_parents order
        }
        const long n = hist[i];
        GroupRule& r = out->rules[i];
        r.slot = k;
        if (dangling[k] >= 0) {                           // any event on k drops its dangling node
            out->rules[dangling[k]].dangle = 0;
            out->kept[k] -= 1;
            dangling[k] = -1;
        }
        if (nmin > 1) {
            const long room = L - tail_fill[k];
            const long keep = n < room ? n : room;
            tail_fill[k] += (int)keep;
            out->kept[k] += keep;
            if (keep < n) {
                r.partial = 1;
                r.keep = (int)keep;
                r.cutoff = 0;                             // set on device when keep > 0
                r.dangle = 1;
                dangling[k] = i;
                out->kept[k] += 1;
            }
        } else {
            out->kept[k] += n;
            tail_fill[k] = (int)((n - 1) % L) + 1;
        }
    }
    for (int i = 0; i < tl; i++) {
        const GroupRule& r = out->rules[i];
        if (r.partial && (r.keep > 0 || r.dangle)) out->search.push_back(i);
    }
    return true;
}

}  // namespace phd
