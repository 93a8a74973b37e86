"""CPU: the C-ABI library loads and exports every symbol include/*.h declares (no compute)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?\w+\s*\*?\s*(mmt_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_entry_points():
    names = _declared()
    assert {"mmt_last_error", "mmt_tome_match", "mmt_tome_merge_wavg_fwd"} <= names


def test_library_exports_every_declared_symbol():
    from multi_modal_transformers_tokenmerge_amd import _C
    lib = ctypes.CDLL(str(_C._LIB_PATH))
    missing = [n for n in sorted(_declared()) if not hasattr(lib, n)]
    assert not missing, f"libmmt_hip.so lacks {missing}"


def test_binding_table_covers_header():
    from multi_modal_transformers_tokenmerge_amd import _C
    assert _declared() <= set(_C.exported_symbols())


def test_version_and_error_without_gpu():
    from multi_modal_transformers_tokenmerge_amd import _C
    assert _C.lib().mmt_version() == _C.API_VERSION == 2
    # argument validation happens before any HIP call: a bad shape returns an error, no abort
    rc = _C.lib().mmt_tome_match(None, 0, 1, 8, 1, 4, 32, 4, 0, 2, 0, None, None, None, None, None,
                                 0, None)
    assert rc == -1 and b"null" in _C.lib().mmt_last_error()


def test_workspace_size_without_gpu():
    from multi_modal_transformers_tokenmerge_amd import _C
    # normalised halves (n t c fp32) + node_max / node_idx (n ceil(t/2) each), 256-B aligned pieces
    n, t, c = 16, 1024, 64
    assert _C.workspace_size(_C.WS_TOME_MATCH, n, t, c) == 4 * n * t * c + 2 * 4 * n * 512
    with pytest.raises(_C.MMTError):
        _C.workspace_size(_C.WS_TOME_MATCH, 1, 8)
    with pytest.raises(_C.MMTError):
        _C.workspace_size(99, 1, 8, 4)
