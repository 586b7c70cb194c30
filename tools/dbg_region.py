"""Stress: region CRC (host scalar hook and device) over random lengths vs the oracle."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc
from tests import _oracle, _prng
vc.init(0)
dev = torch.device("cuda:0")
data = _prng.prng_bytes(5, 1 << 17)
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
G = int(sys.argv[1]) if len(sys.argv) > 1 else 0
vc.set_geometry(G)
lens = rng.integers(2049, 70000, 1500)
want = {int(L): _oracle.crc32(data[:L]) for L in lens}
bad_h, bad_d = [], []
d_all = torch.from_numpy(data).to(dev)
for L in lens:
    L = int(L)
    h = vc.val_crc32(data[:L])
    if h != want[L]:
        bad_h.append(L)
    got = (int(vc.region(d_all[:L]).item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF
    if got != want[L]:
        bad_d.append(L)
print(f"G={G} host bad {len(bad_h)} {bad_h[:10]} dev bad {len(bad_d)} {bad_d[:10]}", flush=True)
