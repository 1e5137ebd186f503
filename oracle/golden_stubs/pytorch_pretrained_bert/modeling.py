"""BertModel with the 0.6.x interface used by src/mmbt.py:90-96,121,124-128, built
from transformers' (independent) BERT modules with random init; weights are then
overwritten from oracle/weights.py by gen_golden.py."""
import torch.nn as nn
from transformers import BertConfig
from transformers.models.bert.modeling_bert import BertEmbeddings, BertEncoder, BertPooler

CONFIG = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
              intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
              attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
              layer_norm_eps=1e-12)


class _Encoder06(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer = BertEncoder(cfg).layer

    def forward(self, hidden, ext_mask, output_all_encoded_layers=True):
        outs = []
        for lyr in self.layer:
            hidden = lyr(hidden, ext_mask)
            hidden = hidden[0] if isinstance(hidden, tuple) else hidden
            outs.append(hidden)
        return outs if output_all_encoded_layers else [hidden]


class BertModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embeddings = BertEmbeddings(cfg)
        self.encoder = _Encoder06(cfg)
        self.pooler = BertPooler(cfg)

    @classmethod
    def from_pretrained(cls, name, **kw):
        cfg = BertConfig(**CONFIG)
        cfg._attn_implementation = "eager"
        return cls(cfg)
