// ASan/UBSan/LSan driver for phd_legacy.cpp (tests/test_legacy_tree.py): the
// legacy report tree is separately malloc'd, so a C caller may free() its
// members (as with the reference, src/interface.c:97-111) and free_full_report's
// tree path frees the rest without a double free or a leak.
#include <cstdio>
#include <cstdlib>

#include "../../include/photohive_dsp.h"

namespace phd {
Full_Report_Data* legacy_tree_copy(const Full_Report_Data* src);
void legacy_tree_free(Full_Report_Data* r);
bool legacy_release(Full_Report_Data* r);
}

static int check(bool ok, const char* what) {
    if (!ok) fprintf(stderr, "FAIL: %s\n", what);
    return ok ? 0 : 1;
}

int main() {
    int bad = 0;
    // 1. members freed by the caller with free(), the rest by the library
    Full_Report_Data* r = phd_debug_legacy_report(7, 72, 40, 3);
    bad += check(r && r->color_palette->N == 7 && r->blur_profile->bins[71][39] == 71 + 0.039, "contents");
    free(r->rgb_stats); r->rgb_stats = nullptr;
    free(r->color_palette->averages); r->color_palette->averages = nullptr;
    free(r->color_palette->percentages); r->color_palette->percentages = nullptr;
    for (int a = 0; a < r->blur_profile->num_angle_bins; a++) {
        free(r->blur_profile->bins[a]);
        r->blur_profile->bins[a] = nullptr;
    }
    free(r->blur_vectors->blur_vectors); r->blur_vectors->blur_vectors = nullptr;
    free(r->blur_vectors); r->blur_vectors = nullptr;
    free(r->sharpness->sharpness); r->sharpness->sharpness = nullptr;
    bad += check(phd::legacy_release(r), "release of a live tree");
    // 2. a tree released twice: the second call is ignored (not a live tree)
    Full_Report_Data* r2 = phd_debug_legacy_report(0, 1, 1, -1);
    bad += check(r2 && r2->sharpness == nullptr && r2->color_palette->N == 0, "empty shape");
    bad += check(phd::legacy_release(r2), "release");
    bad += check(!phd::legacy_release(r2), "second release ignored");
    // 3. a copy of a stack tree, freed whole (the reference's free order)
    Full_Report_Data* r3 = phd_debug_legacy_report(64, 256, 256, 64);
    Full_Report_Data* r4 = phd::legacy_tree_copy(r3);
    bad += check(r4 && r4->blur_profile->bins[255][255] == r3->blur_profile->bins[255][255], "copy");
    phd::legacy_tree_free(r4);
    bad += check(phd::legacy_release(r3), "release r3");
    if (!bad) printf("legacy tree OK\n");
    return bad;
}
