"""The C-ABI library loads and exports every symbol include/kdstep.h declares (CPU only)."""
import ctypes

import pytest

from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as N


def test_library_loads_and_version():
    lib = N.lib()
    assert lib.kd_abi_version() == 1
    assert isinstance(lib.kd_last_error(), bytes)


def test_every_header_symbol_is_exported():
    names = N.header_symbols()
    assert len(names) >= 6
    raw = ctypes.CDLL(str(N.LIB_PATH))
    missing = [n for n in names if not hasattr(raw, n)]
    assert not missing, f"declared in include/kdstep.h but not exported: {missing}"
    # and the Python binding covers every declared symbol
    assert set(names) == set(N.SIGNATURES), set(names) ^ set(N.SIGNATURES)


def test_status_codes_raise_with_message():
    lib = N.lib()
    # argument validation happens before any device call: null pointers -> KD_ERR_ARG
    prm = N.KdLossParams(N.KD_LOSS_LOCA, 1.0, 0.8, 1.0, 1.0, 1.0, 1e-8, 1)
    st = lib.kd_loss_fwd_bwd(None, 0, 0, None, 0, 0, None, 1, 1, prm, None, None, 0, None, 0, None)
    assert st == 7
    assert b"null" in lib.kd_last_error()
    with pytest.raises(N.KdError):
        N.check("kd_loss_fwd_bwd", st)


def test_workspace_size_grows_with_shape():
    lib = N.lib()
    assert lib.kd_loss_workspace_size(4, 1536, 151936) > lib.kd_loss_workspace_size(1, 1536, 151936)
