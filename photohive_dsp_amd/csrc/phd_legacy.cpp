// phd_legacy.cpp -- reports for the reference's C callers in the reference's
// own allocation shape.
//
// get_full_report_data (src/interface.c:20-94) returns a tree in which every
// structure and array is its own malloc: compile_full_report's members,
// Color_Palette's averages / percentages (free_color_palette,
// src/color_quantization.c:614-618), the blur profile's row-pointer array and
// each of its rows (free_blur_profile + free_2d_array, src/blur_profile.c:
// 473-478, src/utilities.c:181-186), the vector group and its vectors
// (free_blur_vector_group, src/blur_profile.c:481-484) and the sharpnesses
// (src/interface.c:103-106).  A C caller may therefore free() any member
// itself.  The batch entry points keep one pooled block per report
// (phd_report.cpp, assemble); the legacy entry copies that block into such a
// tree, and free_full_report (src/interface.c:97-111) frees a tree member by
// member.  Host-only C++ (no HIP), so tests/test_legacy_tree.py builds it
// with a sanitiser on the CPU.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_set>

#include "../../include/photohive_dsp.h"

namespace phd {

namespace {

struct LegacySet {
    std::mutex m;
    std::unordered_set<const void*> live;   // trees handed out by the legacy entry
};
LegacySet& legacy_set() {
    static LegacySet* s = new LegacySet;    // process lifetime: reports may be freed at exit
    return *s;
}

template <class T>
T* dup_array(const T* src, size_t n) {      // n >= 1 elements, so the result is never a NULL "empty"
    const size_t k = n ? n : 1;
    T* d = static_cast<T*>(malloc(sizeof(T) * k));
    if (d) {
        memset(d, 0, sizeof(T) * k);
        if (src && n) memcpy(d, src, sizeof(T) * n);
    }
    return d;
}

}  // namespace

// Frees a tree member by member, as src/interface.c:97-111 does, tolerating
// members a caller has already freed and set to NULL.
void legacy_tree_free(Full_Report_Data* r) {
    if (!r) return;
    if (Color_Palette* cp = r->color_palette) {
        free(cp->averages);
        free(cp->percentages);
        free(cp);
    }
    if (Blur_Profile* bp = r->blur_profile) {
        if (bp->bins) {
            for (int a = 0; a < bp->num_angle_bins; a++) free(bp->bins[a]);
            free(bp->bins);
        }
        free(bp);
    }
    if (Blur_Vector_Group* bv = r->blur_vectors) {
        free(bv->blur_vectors);
        free(bv);
    }
    if (Sharpnesses* sh = r->sharpness) {
        free(sh->sharpness);
        free(sh);
    }
    free(r->rgb_stats);
    free(r);
}

// A separately allocated copy of report `src` (any layout), or nullptr when an
// allocation fails (nothing is leaked then).
Full_Report_Data* legacy_tree_copy(const Full_Report_Data* src) {
    if (!src) return nullptr;
    Full_Report_Data* r = static_cast<Full_Report_Data*>(calloc(1, sizeof(Full_Report_Data)));
    if (!r) return nullptr;
    bool ok = true;
    r->average_saturation = src->average_saturation;
    if (src->rgb_stats) ok &= (r->rgb_stats = dup_array(src->rgb_stats, 1)) != nullptr;
    if (const Color_Palette* s = src->color_palette) {
        Color_Palette* cp = static_cast<Color_Palette*>(calloc(1, sizeof(Color_Palette)));
        r->color_palette = cp;
        if (cp) {
            cp->N = s->N;
            const size_t n = s->N > 0 ? (size_t)s->N : 0;
            ok &= (cp->averages = dup_array(s->averages, n)) != nullptr;
            ok &= (cp->percentages = dup_array(s->percentages, n)) != nullptr;
        } else {
            ok = false;
        }
    }
    if (const Blur_Profile* s = src->blur_profile) {
        Blur_Profile* bp = static_cast<Blur_Profile*>(calloc(1, sizeof(Blur_Profile)));
        r->blur_profile = bp;
        if (bp) {
            *bp = *s;
            bp->bins = nullptr;
            const int na = s->num_angle_bins > 0 ? s->num_angle_bins : 0;
            const size_t nr = s->num_radius_bins > 0 ? (size_t)s->num_radius_bins : 0;
            Bin** rows = static_cast<Bin**>(calloc(na ? (size_t)na : 1, sizeof(Bin*)));
            if (rows) {
                bp->bins = rows;
                for (int a = 0; a < na; a++) ok &= (rows[a] = dup_array(s->bins ? s->bins[a] : nullptr, nr)) != nullptr;
            } else {
                bp->num_angle_bins = 0;
                ok = false;
            }
        } else {
            ok = false;
        }
    }
    if (const Blur_Vector_Group* s = src->blur_vectors) {
        Blur_Vector_Group* bv = static_cast<Blur_Vector_Group*>(calloc(1, sizeof(Blur_Vector_Group)));
        r->blur_vectors = bv;
        if (bv) {
            bv->len_vectors = s->len_vectors;
            ok &= (bv->blur_vectors = dup_array(s->blur_vectors, s->len_vectors > 0 ? (size_t)s->len_vectors : 0)) !=
                  nullptr;
        } else {
            ok = false;
        }
    }
    if (const Sharpnesses* s = src->sharpness) {
        Sharpnesses* sh = static_cast<Sharpnesses*>(calloc(1, sizeof(Sharpnesses)));
        r->sharpness = sh;
        if (sh) {
            sh->N = s->N;
            ok &= (sh->sharpness = dup_array(s->sharpness, s->N > 0 ? (size_t)s->N : 0)) != nullptr;
        } else {
            ok = false;
        }
    }
    if (!ok) {
        legacy_tree_free(r);
        return nullptr;
    }
    return r;
}

void legacy_register(const Full_Report_Data* r) {
    LegacySet& s = legacy_set();
    std::lock_guard<std::mutex> lk(s.m);
    s.live.insert(r);
}

// true (and the tree freed) when r is a live legacy tree; false, nothing read
// or freed, otherwise
bool legacy_release(Full_Report_Data* r) {
    LegacySet& s = legacy_set();
    {
        std::lock_guard<std::mutex> lk(s.m);
        if (!s.live.erase(r)) return false;
    }
    legacy_tree_free(r);
    return true;
}

}  // namespace phd

// Test hook (tests/test_legacy_tree.py and the ASan driver in tools/): a tree
// of the given shape, filled with a recognisable pattern, registered as a live
// legacy report -- what get_full_report_data returns, without a GPU.
extern "C" Full_Report_Data* phd_debug_legacy_report(int n_palette, int na, int nr, int n_crops) {
    Pixel_HSV avg[64];
    double pct[64];
    const int np = n_palette < 0 ? 0 : (n_palette > 64 ? 64 : n_palette);
    for (int k = 0; k < np; k++) {
        avg[k] = Pixel_HSV{k, 1.0 * k, 0.5, 0.25};
        pct[k] = 0.01 * k;
    }
    Color_Palette cp{np, avg, pct};
    const int a_n = na < 0 ? 0 : (na > 256 ? 256 : na), r_n = nr < 0 ? 0 : (nr > 256 ? 256 : nr);
    static thread_local Bin rowbuf[256 * 256];
    Bin* rowp[256];
    for (int a = 0; a < a_n; a++) {
        rowp[a] = rowbuf + (size_t)a * r_n;
        for (int q = 0; q < r_n; q++) rowp[a][q] = a + 0.001 * q;
    }
    Blur_Profile bp{a_n, r_n, 5, 7, rowp};
    Blur_Vector vec[10];
    for (int k = 0; k < 10; k++) vec[k] = Blur_Vector{k, 0.5f * k};
    Blur_Vector_Group bv{10, vec};
    double shv[64];
    const int nc = n_crops < 0 ? -1 : (n_crops > 64 ? 64 : n_crops);
    for (int k = 0; k < 64; k++) shv[k] = 2.0 * k;
    Sharpnesses sh{nc, shv};
    RGB_Statistics st{0.1, 0.2, 0.3, 0.4, 0.5, 0.6};
    Full_Report_Data src{&st, &cp, &bp, &bv, 0.75, nc >= 0 ? &sh : nullptr};
    Full_Report_Data* r = phd::legacy_tree_copy(&src);
    if (r) phd::legacy_register(r);
    return r;
}
