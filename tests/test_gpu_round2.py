"""GPU tests added in round 2: determinism of the blur bins, stream ordering with
PyTorch producers, and batched runtime-plan sizes with downsample_rate > 1.

Every test calls through the C-ABI (libreport_data.so); the oracle is only
the checker.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _phd():
    import torch
    import photohive_dsp_amd as phd
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return phd, torch


def _bins(rep):
    return np.array(rep.blur_profile.bins)


@pytest.mark.parametrize("kind,h,w", [("structured", 3000, 4000), ("symmetric", 512, 512), ("hblur", 720, 1280)])
def test_blur_bins_bit_identical_over_repeats(kind, h, w):
    """vectorize_blur_profile (src/blur_profile.c:324-416) thresholds the bins with
    strict comparisons, so they must not move between runs: the column pass sums
    them as fixed-point integers (order-independent atomics).  10 runs of the same
    image in one process give bit-identical bins and vectors."""
    phd, torch = _phd()
    from photohive_dsp_amd import synth
    if kind == "symmetric":
        # mirror-symmetric in both axes: many exactly equal bins and ties
        q = synth.structured(h // 2, w // 2, 9)
        img = np.ascontiguousarray(np.concatenate([np.concatenate([q, q[:, ::-1]], 1),
                                                   np.concatenate([q[::-1], q[::-1, ::-1]], 1)], 0))
    else:
        img = synth.make(kind, h, w, 31)
    t = torch.from_numpy(img).cuda()[None].contiguous()
    first = phd.report_device(t)[0]
    b0, v0 = _bins(first), [(v.angle, v.magnitude) for v in first.blur_vectors]
    for _ in range(9):
        r = phd.report_device(t)[0]
        assert np.array_equal(_bins(r), b0)
        assert [(v.angle, v.magnitude) for v in r.blur_vectors] == v0
    # the host-buffer path gives the same bits
    r = phd.get_report(img)
    assert np.array_equal(_bins(r), b0)


def test_device_input_produced_by_async_torch_op():
    """A device image still being produced on PyTorch's (null) stream when the
    call is made: the library orders its stream after it (work_stream)."""
    phd, torch = _phd()
    from photohive_dsp_amd import synth
    img = synth.structured(600, 800, 5)
    src = torch.from_numpy(img).cuda()
    torch.cuda.synchronize()
    a = torch.randn(6144, 6144, device="cuda")
    for _ in range(4):
        a = a @ a                                   # keeps the stream busy for milliseconds
        a = a / a.abs().max()
    t = (src.to(torch.int16) + (a[0, 0] * 0).to(torch.int16)).to(torch.uint8)[None].contiguous()
    r = phd.report_device(t)[0]
    ref = phd.get_report(img)
    assert r.color_palette.group_ids == ref.color_palette.group_ids
    assert r.color_palette.quantities == ref.color_palette.quantities
    assert np.array_equal(_bins(r), _bins(ref))


@pytest.mark.parametrize("shape", [(512, 512), (513, 700)])
def test_batched_runtime_plan_with_downsample(shape):
    """Two same-size images without a compile-time FFT plan at downsample_rate 2:
    the batched row pass reads the device pointer array, which must be uploaded
    on this path too (it used to be stale).  Each report equals the single-image
    report and the oracle."""
    phd, torch = _phd()
    from oracle import oracle as orc
    from photohive_dsp_amd import synth
    h, w = shape
    imgs = [synth.make("structured", h, w, 61), synth.make("uniform", h, w, 62)]
    reps = phd.get_reports(imgs, downsample_rate=2)
    for img, r in zip(imgs, reps):
        one = phd.get_report(img, downsample_rate=2)
        assert r.color_palette.group_ids == one.color_palette.group_ids
        assert r.color_palette.quantities == one.color_palette.quantities
        assert np.array_equal(_bins(r), _bins(one))
        o = orc.report(img, downsample_rate=2)
        np.testing.assert_array_equal(np.array(r.color_palette.group_ids), o.valid_parents)
        np.testing.assert_array_equal(np.array(r.color_palette.quantities), o.palette_pct)
        np.testing.assert_allclose(_bins(r), o.bins, rtol=1e-4, atol=1e-12)


def test_host_batch_pipelined_groups_match_device_reports():
    """phd_report_batch_u8 with several same-size groups (16 + 4 + 3 images):
    the uploads go through the pinned slot ring while the previous group
    computes; every report equals the device-resident report of its image."""
    phd, torch = _phd()
    from photohive_dsp_amd import synth
    imgs = [synth.make(("uniform", "structured", "hblur")[i % 3], 480, 640, 200 + i) for i in range(20)]
    imgs += [synth.make("structured", 512, 512, 300 + i) for i in range(3)]
    order = list(range(0, 23, 2)) + list(range(1, 23, 2))          # interleave the sizes
    imgs = [imgs[i] for i in order]
    reps = phd.get_reports(imgs)
    for img, r in zip(imgs, reps):
        one = phd.report_device(torch.from_numpy(img).cuda()[None].contiguous())[0]
        assert r.color_palette.group_ids == one.color_palette.group_ids
        assert r.color_palette.quantities == one.color_palette.quantities
        assert np.array_equal(_bins(r), _bins(one))
        assert [v.angle for v in r.blur_vectors] == [v.angle for v in one.blur_vectors]


def test_two_lanes_match_one_lane():
    """phd_set_lanes(2): a device batch of >= 16 images is split over two
    contexts (the second half on the library's lane thread).  Every report
    equals the one-lane report of the same batch, field by field, and a failing
    second half would surface through the status array."""
    phd, torch = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.lib import lib
    imgs = [synth.make(("uniform", "structured", "hblur")[i % 3], 600, 800, 400 + i) for i in range(20)]
    t = torch.from_numpy(np.stack(imgs)).cuda().contiguous()
    prev = lib.phd_set_lanes(1)
    try:
        one = phd.report_device(t)
        assert lib.phd_set_lanes(2) == 1
        two = phd.report_device(t)
        two_again = phd.report_device(t)
    finally:
        lib.phd_set_lanes(prev)
    for a, b, c in zip(one, two, two_again):
        for r in (b, c):
            assert r.color_palette.group_ids == a.color_palette.group_ids
            assert r.color_palette.quantities == a.color_palette.quantities
            assert np.array_equal(_bins(r), _bins(a))
            assert [(v.angle, v.magnitude) for v in r.blur_vectors] == \
                [(v.angle, v.magnitude) for v in a.blur_vectors]
            # fp64 sums from atomics: order-dependent in the last bits on either lane count
            assert r.average_saturation == pytest.approx(a.average_saturation, rel=1e-12)
            for f in ("Br", "Bg", "Bb", "Cr", "Cg", "Cb"):
                assert getattr(r.rgb_stats, f) == pytest.approx(getattr(a.rgb_stats, f), rel=1e-12)


def test_concurrent_callers_with_lanes():
    """Two host threads call report_device at once with 16-image batches (lanes
    on): one gets the lane worker, the other runs its whole batch on lane 0
    (the worker is never waited for); no deadlock, and every report equals the
    one-lane report of its image."""
    import threading
    phd, torch = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.lib import lib
    imgs = [synth.make(("uniform", "structured")[i % 2], 480, 640, 700 + i) for i in range(16)]
    t = torch.from_numpy(np.stack(imgs)).cuda().contiguous()
    prev = lib.phd_set_lanes(1)
    try:
        ref = phd.report_device(t)
        lib.phd_set_lanes(2)
        out, errs = [None, None], []

        def work(k):
            try:
                out[k] = phd.report_device(t)
            except Exception as e:        # surfaced below
                errs.append(e)
        th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=60)
        assert not any(x.is_alive() for x in th), "a caller is stuck"
        assert not errs, errs
    finally:
        lib.phd_set_lanes(prev)
    for reps in out:
        for a, r in zip(ref, reps):
            assert r.color_palette.group_ids == a.color_palette.group_ids
            assert r.color_palette.quantities == a.color_palette.quantities
            assert np.array_equal(_bins(r), _bins(a))
