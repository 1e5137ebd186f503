"""CPU: the C-ABI library loads, exports every entry point include/mmu.h declares, and
the Python binding declares exactly those (no compute calls -- no GPU here)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mmu.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mmu_\w+)\s*\(", txt)))


def test_header_declares_the_api():
    names = declared()
    for must in ("mmu_gemm", "mmu_attention_fwd", "mmu_attention_bwd", "mmu_layernorm_fwd", "mmu_layernorm_bwd",
                 "mmu_embed_fwd", "mmu_embed_bwd", "mmu_bertadam_step", "mmu_uncertainty", "mmu_ece_bins",
                 "mmu_last_error", "mmu_version"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from src import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libmmu_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared()) == set(_native.SIGNATURES), "binding table and header disagree"
    assert _native.load().mmu_version() == 4


def test_epilogue_struct_layout_matches_header(tmp_path):
    """ctypes mirror vs the C compiler's layout of mmu_epilogue (sizeof + every offsetof)."""
    import shutil
    import subprocess
    from src._native import Epilogue
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    fields = [f for f, _ in Epilogue._fields_]
    src = tmp_path / "lay.c"
    body = "".join(f'printf("%zu\\n", offsetof(mmu_epilogue, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\n'
                   f'int main(void){{printf("%zu\\n", sizeof(mmu_epilogue));{body}return 0;}}\n')
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    out = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    assert out[0] == ctypes.sizeof(Epilogue)
    assert out[1:] == [getattr(Epilogue, f).offset for f in fields]


def test_kernels_refuse_cpu_tensors():
    import torch
    from src import kernels as K
    from src._native import NativeError
    a = torch.zeros(128, 64, dtype=torch.bfloat16)
    with pytest.raises(NativeError, match="HIP"):
        K.gemm(a, 64, True, a, 64, True, torch.zeros(128, 128), 128, 128, 128, 64)


def test_model_has_no_cpu_fallback():
    import torch
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args, synthetic_batch
    from src._native import NativeError
    m = MultimodalBertClf(small_args())
    x, _ = synthetic_batch(1, 4, vocab=4096)
    with pytest.raises(NativeError):
        m(*x)
