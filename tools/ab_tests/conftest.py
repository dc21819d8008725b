"""The A/B tests run the tools' A/B library (tools/ab/libkdstep_ab.so: the product sources built
with -DKD_AB_BUILD, i.e. also the negative-result / diagnostic kernels and the ab_knob switches),
loaded through KDSTEP_LIB before the package binds its library."""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent.parent
AB_LIB = REPO / "tools" / "ab" / "libkdstep_ab.so"
os.environ.setdefault("KDSTEP_LIB", str(AB_LIB))
# v8's k-loop stagger (GemmP.stagger, on in the product) changes v8's summation order; the A/B
# kernels (v9, v11, v12) have none, so their bit-exact comparisons run v8 unstaggered. The A/B
# library reads the switch on every launch: test_v8_stagger_* turns it on where it compares.
os.environ.setdefault("KD_GEMM_STAGGER", "0")
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "tests" / "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def pytest_collection_modifyitems(config, items):
    import torch
    why = None
    if not torch.cuda.is_available():
        why = "no GPU in this container"
    elif not Path(os.environ["KDSTEP_LIB"]).exists():
        why = f"A/B library not built: {os.environ['KDSTEP_LIB']} (csrc/build.py --ab)"
    if why:
        for it in items:
            it.add_marker(pytest.mark.skip(reason=why))


@pytest.fixture(scope="session")
def dev():
    import torch
    return torch.device("cuda:0")
