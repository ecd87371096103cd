"""The skewed wave partition (wave_range, open-rdma-driver_amd/csrc/icrc_device.h), restated:
for every skew the defaults and the A/B sweeps use, the 16 waves' ranges tile the workgroup's
16 x chunk packets exactly, in whole units, ordered oldest-first; with the product's defaults no
wave is left empty (the kernels also accept an empty range: its wave only joins the table fill)."""
import pytest


def wave_range(g0, chunk, wave, skew):
    unit = 8 << ((skew >> 12) & 3)
    e = skew & 0xFFF
    if e == 0 or chunk < 64:
        return g0 + wave * chunk, g0 + wave * chunk + chunk
    U = 16 * chunk // unit

    def start(k):
        f, r = k >> 2, k & 3
        return U * (1024 * k + e * (4 * f * (4 - f) + r * (3 - 2 * f))) // (16 * 1024)
    return g0 + unit * start(wave), g0 + unit * start(wave + 1)


@pytest.mark.parametrize("skew", [0, 45, 45 | 3 << 12, 135 | 3 << 12, 180, 300])
@pytest.mark.parametrize("chunk", [8, 64, 256, 1024, 4096])
def test_ranges_tile_the_workgroup(skew, chunk):
    g0 = 7 * 16 * chunk
    r = [wave_range(g0, chunk, k, skew) for k in range(16)]
    assert r[0][0] == g0 and r[-1][1] == g0 + 16 * chunk
    assert all(r[k][1] == r[k + 1][0] for k in range(15))
    unit = 8 << ((skew >> 12) & 3) if (skew & 0xFFF) and chunk >= 64 else 1
    assert all((hi - lo) % unit == 0 and hi >= lo for lo, hi in r)  # an empty wave only returns
    if skew in (45 | 3 << 12, 180):  # the product's defaults (kWaveSkewOct, kWaveSkewLong): no empty wave
        assert all(hi > lo for lo, hi in r)
    if skew & 0xFFF and chunk >= 1024:  # enough units for the shares to order by age
        by_age = [sum(r[k][1] - r[k][0] for k in range(16) if k >> 2 == a) for a in range(4)]
        assert by_age == sorted(by_age, reverse=True)
