"""GF(2) combine/shift of the product library (host-side math, no GPU)
against the reference-derived combine triples and the oracle."""
import numpy as np

import val_protocol_amd.crc as vc
from tests import _oracle


def test_combine_matches_reference_triples(golden):
    for la, lb, ca, cb, cab in golden["combine"]:
        assert vc.crc32_combine(ca, cb, lb) == cab


def test_shift_matches_oracle():
    rng = np.random.default_rng(1)
    for _ in range(200):
        st = int(rng.integers(0, 2**32))
        n = int(rng.integers(0, 2**40))
        assert vc.crc32_shift(st, n) == _oracle.shift(st, n)
    assert vc.crc32_shift(0x12345678, 0) == 0x12345678


def test_init_finalize():
    assert vc.val_crc32_init_state() == 0xFFFFFFFF
    assert vc.val_crc32_finalize_state(0xFFFFFFFF) == 0
