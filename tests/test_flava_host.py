"""CPU: the FLAVA drop-in (src/model.py) exposes the reference's module tree / state_dict keys
(so reference checkpoints load strictly) and refuses to compute without the HIP path."""
import json
import os

import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("tag,kw", [("vanilla", dict(out_dim=1)), ("multihead_avgpool", dict(out_dim=2, avg_pool=True)),
                                    ("cls_multihead", dict(out_dim=2, clstoken=True))])
def test_state_dict_keys_match_reference(tag, kw):
    from src.model import FlavaFusionTransfomer, FlavaFusionTransfomerwithCLSToken
    from oracle import flava_ref as FR
    cls = FlavaFusionTransfomerwithCLSToken if kw.get("clstoken") else FlavaFusionTransfomer
    m = cls(out_dim=kw["out_dim"], num_classes=2, avg_pool=kw.get("avg_pool", False), drop=0.0)
    ref = json.load(open(os.path.join(GOLD, f"flava_{tag}_keys.json")))
    assert list(m.state_dict().keys()) == ref["state_dict_keys"]
    assert [n for n, _ in m.named_parameters()] == ref["named_parameters"]
    m.load_state_dict(FR.make_state_dict(0, FR.FlavaConfig(**kw)), strict=True)


def test_mlp_is_four_modules_like_the_reference():
    """The reference's OrderedDict repeats "dropout": c_fc, dropout, gelu, c_proj."""
    from src.model import ResidualAttentionBlock
    b = ResidualAttentionBlock(768, 3, drop=0.3)
    assert list(b.mlp._modules) == ["c_fc", "dropout", "gelu", "c_proj"]


def test_flava_refuses_cpu_tensors():
    from src.model import FlavaFusionTransfomer
    from src._native import NativeError
    m = FlavaFusionTransfomer(out_dim=1, num_classes=2, avg_pool=False)
    with pytest.raises(NativeError):
        m((torch.randn(2, 3, 768), torch.randn(2, 4, 768)))
