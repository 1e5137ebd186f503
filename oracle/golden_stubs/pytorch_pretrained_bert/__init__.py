"""pytorch_pretrained_bert 0.6.x stand-in (see ../README.md)."""
