// Host cost of decide_palette (find_valid_octree_parents + group_irregular_pixels
// as keep rules) on a saved group histogram, and a randomized check that the
// fast paths (contiguous insertion scan, nearest-order table) decide exactly
// as custom_sort's swap-by-swap insertion sort and the all-parents search.
// Build:
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/decide_bench.cpp \
//       build/obj/*.o -L/opt/rocm/lib -lamdhip64 -o /tmp/decide_bench
// Usage: decide_bench hist.bin h s v [iters]
#include <chrono>
#include <climits>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../photohive_dsp_amd/csrc/phd_host.h"

using namespace phd;

static bool same(const PaletteDecision& a, const PaletteDecision& b) {
    if (a.parents != b.parents || a.kept != b.kept || a.search != b.search || a.rules.size() != b.rules.size())
        return false;
    for (size_t g = 0; g < a.rules.size(); g++)
        if (memcmp(&a.rules[g], &b.rules[g], sizeof(GroupRule))) return false;
    return true;
}

// custom_sort (src/utilities.c:132-153) swap by swap: the parents prefix
static std::vector<int> slow_order(const GridParams& g, const GroupCenters& gc, const unsigned* hist,
                                   const phd_config& cfg) {
    std::vector<float> sal(g.tl);
    for (int i = 0; i < g.tl; i++) {
        const float s_v = (float)(gc.s[i] * gc.v[i]);
        sal[i] = (float)(int)hist[i] * (cfg.quantity_weight + cfg.saturation_value_weight * s_v) * 1000;
    }
    auto cmp = [](float a, float b) {
        const float d = b - a;
        if (!(d > -2147483648.0f && d < 2147483648.0f)) return INT_MIN;
        return (int)d;
    };
    std::vector<int> o(g.tl);
    for (int i = 0; i < g.tl; i++) o[i] = i;
    for (int i = 1; i < g.tl; i++)
        for (int j = i; j > 0 && cmp(sal[o[j]], sal[o[j - 1]]) < 0; j--) std::swap(o[j], o[j - 1]);
    return o;
}

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<unsigned> hist(8192);
    const size_t n = fread(hist.data(), 4, hist.size(), f);
    fclose(f);
    phd_config cfg;
    phd_config_default(&cfg);
    cfg.h_partitions = atoi(argv[2]);
    cfg.s_partitions = atoi(argv[3]);
    cfg.v_partitions = atoi(argv[4]);
    const int iters = argc > 5 ? atoi(argv[5]) : 200;
    const GridParams gp = make_grid(cfg);
    const GroupCenters gc = make_centers(gp);
    if ((size_t)gp.tl != n) fprintf(stderr, "hist has %zu groups, grid %d\n", n, gp.tl);
    auto t0 = std::chrono::steady_clock::now();
    const std::vector<uint16_t> near = make_near_order(gp, gc);
    auto t1 = std::chrono::steady_clock::now();
    printf("near-order table: %.1f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
    long tot = 0;
    for (int g = 0; g < gp.tl; g++) tot += hist[g];
    PaletteDecision d, e;
    for (int mode = 0; mode < 2; mode++) {
        const uint16_t* nr = mode && !near.empty() ? near.data() : nullptr;
        t0 = std::chrono::steady_clock::now();
        for (int it = 0; it < iters; it++)
            if (!decide_palette(gp, gc, hist.data(), tot, cfg, mode ? &e : &d, nr)) return 1;
        t1 = std::chrono::steady_clock::now();
        printf("%s: parents %zu search %zu  %.1f us/decision\n", mode ? "near table" : "all parents",
               d.parents.size(), d.search.size(),
               std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
    }
    if (getenv("DUMP_RULES"))                           // partial groups: g keep dangle
        for (int g : d.search) printf("rule %d %d %d\n", g, d.rules[g].keep, d.rules[g].dangle);
    if (!same(d, e)) {
        printf("MISMATCH on the saved histogram\n");
        return 1;
    }
    // randomized: sparse / dense / huge counts (compare's INT_MIN side), ties
    std::mt19937_64 rng(12345);
    int checked = 0;
    for (int t = 0; t < 400; t++) {
        std::vector<unsigned> h(gp.tl);
        const int mode = t % 4;
        long s = 0;
        for (int g = 0; g < gp.tl; g++) {
            unsigned v = 0;
            if (mode == 0) v = (unsigned)(rng() % 50);
            else if (mode == 1) v = (rng() % 4 == 0) ? (unsigned)(rng() % 100000) : 0;
            else if (mode == 2) v = (unsigned)(rng() % 3) * 7;
            else v = (rng() % 8 == 0) ? (unsigned)(rng() % 30000000) : (unsigned)(rng() % 3);
            h[g] = v;
            s += v;
        }
        if (s == 0) continue;
        PaletteDecision a, b;
        const bool oa = decide_palette(gp, gc, h.data(), s, cfg, &a, nullptr);
        const bool ob = decide_palette(gp, gc, h.data(), s, cfg, &b, near.empty() ? nullptr : near.data());
        if (oa != ob || (oa && !same(a, b))) {
            printf("MISMATCH near vs all-parents, trial %d\n", t);
            return 1;
        }
        if (oa) {
            const std::vector<int> o = slow_order(gp, gc, h.data(), cfg);
            if (!std::equal(a.parents.begin(), a.parents.end(), o.begin())) {
                printf("MISMATCH insertion order, trial %d\n", t);
                return 1;
            }
        }
        checked++;
    }
    printf("randomized: %d histograms identical\n", checked);
    return 0;
}
