"""Host-side checks of the SSD front end (no GPU needed)."""
import pytest

from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.ssd import _spec_of, compute_ssd_hist


def test_spec_lookup_and_size_limit():
    spec = EnvSpec(load_network("pbn70"), [])
    assert _spec_of(spec) is spec

    class Wrapper:   # gymnasium-style env.env chain
        def __init__(self, inner):
            self.env = inner

    class Holder:
        def __init__(self, s):
            self.spec = s

    assert _spec_of(Wrapper(Holder(spec))) is spec
    with pytest.raises(ValueError, match="at most 32 nodes"):
        compute_ssd_hist(spec, resets=32, iters=1)
    with pytest.raises(TypeError):
        _spec_of(object())


def test_bittner28_histogram_fits_hbm():
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    assert (1 << spec.n) * 4 == 1 << 30   # 1 GiB of 32-bit counters
