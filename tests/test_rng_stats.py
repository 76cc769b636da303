"""Statistical check of the Tier-B counter RNG (VERDICT r4 ask 1).

The reference renders with one sequential Xoshiro256++ stream (main.zig:300,
rand.zig:13-40) that no parallel renderer can reproduce, so the GPU contract's
generator only has to behave as independent uniform words in the relations a
render uses.  tests/native/rng_stats.c measures exactly those over 2^32 draws
laid out as a render lays them out (2^16 pixels x 2^8 samples x 2^8 draws of
the Weyl blocks of oracle/rtw_oracle.c tierb_state): bit bias, byte
uniformity, lag-1 pairs on every byte, lag-2/3 pairs, triples (the unit-ball
candidate), Hamming-weight dependency, and every byte of the same draw of
neighbouring samples and of neighbouring pixels (p+1, p+W), plus Pearson
correlations of the reals.  The mixer it tests is checked to be the oracle's
ro_tb_mix word for word, and a control mixer that is known to be weak must
fail the same battery (the battery has teeth)."""
import ctypes as C
import json
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "rng_stats.c")
CONTRACT_MIXER = 10  # rng_stats.c numbering of the Tier-B mixer (four Feistel half-rounds)


@pytest.fixture(scope="module")
def battery(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rng") / "rng_stats")
    subprocess.run(["gcc", "-O3", "-march=native", "-fopenmp", "-o", exe, SRC, "-lm"], check=True)
    return exe


def run(exe, mixer, lp, ls, lk, limit=5.0):
    r = subprocess.run([exe, str(mixer), str(lp), str(ls), str(lk), str(limit)], capture_output=True, text=True)
    assert r.returncode in (0, 1), r.stderr
    return json.loads(r.stdout)


def test_battery_tests_the_oracle_mixer(battery, oracle):
    L = oracle.lib()
    rnd = random.Random(11)
    for x in [0, 1, (1 << 64) - 1, L.ro_tierb_state(42, 0, 0)] + [rnd.getrandbits(64) for _ in range(20)]:
        out = subprocess.run([battery, "dump", str(CONTRACT_MIXER), str(x)], capture_output=True, text=True,
                             check=True).stdout
        assert int(out) == L.ro_tb_mix(C.c_uint64(x)), hex(x)


def test_weak_control_mixer_fails(battery):
    """One multiply between two 32-bit folds: neighbouring pixels (same low
    Weyl word) stay correlated; the battery must reject it at 2^26 draws."""
    d = run(battery, 2, 12, 6, 8)
    assert not d["pass"] and d["pix1_bytes_max_z"] > 20, d


def test_tierb_mixer_passes_2p32_draws(battery):
    d = run(battery, CONTRACT_MIXER, 16, 8, 8)
    print(json.dumps(d))
    assert d["draws"] == 2 ** 32
    assert d["pass"], d
    for k in ("corr_lag1", "corr_samp", "corr_pix"):
        assert abs(d[k]) < 1e-3, (k, d[k])
    assert abs(d["mean"] - 0.5) < 1e-4
