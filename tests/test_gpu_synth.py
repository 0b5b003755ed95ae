"""Device workload generators (include/cs_synth.h) against the oracle's host
generators (oracle/fm_oracle.c): the bench's synthetic text and Q_text / Q_unif
batches are the SURVEY.md §8(d) streams, bit for bit."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import load_pkg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["dna", "bytes", "rdna"])
def test_text_and_patterns(kind):
    pkg = load_pkg()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    L = 100_003 if kind != "rdna" else 3_000_017  # rdna: past two copies of its seed sequence
    text = torch.empty(L + 1 + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device(kind, 42, L, text.data_ptr(), st)
    want = {"dna": O.gen_dna, "bytes": O.gen_bytes, "rdna": O.gen_rdna}[kind](42, L)
    torch.cuda.synchronize()
    host = text[: L + 1].cpu().numpy()
    assert np.array_equal(host, want)
    m, npat, first = 8 if kind == "bytes" else 20, 5000, 0
    pats = torch.empty(npat * m, dtype=torch.uint8, device=dev)
    offs = torch.empty(npat + 1, dtype=torch.int64, device=dev)
    pkg.synth_patterns_device(text.data_ptr(), L + 1, m, first, npat, 4242, pats.data_ptr(),
                              offs.data_ptr(), st)
    torch.cuda.synchronize()
    assert np.array_equal(pats.cpu().numpy().reshape(npat, m), O.gen_patterns_text(want, m, npat))
    assert offs.cpu().numpy().tolist() == list(range(0, (npat + 1) * m, m))


@pytest.mark.parametrize("kind,m", [("dna", 20), ("dna", 70), ("bytes", 8), ("bytes", 19)])
def test_unif_patterns(kind, m):
    pkg = load_pkg()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    npat, first = 3000, 777
    pats = torch.empty(npat * m, dtype=torch.uint8, device=dev)
    pkg.synth_random_patterns_device(kind, m, first, npat, 4242, pats.data_ptr(), None, st)
    torch.cuda.synchronize()
    want = O.gen_patterns_unif(kind, m, first + npat)[first:]
    assert np.array_equal(pats.cpu().numpy().reshape(npat, m), want)
