"""CPU oracle for the MMBT hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in the product (``multi-modal-uncertainty_amd/``) may import this
package.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / the timed CPU baseline.

Contents
--------
weights.py        seeded init recipe producing a state_dict whose keys are the
                  reference ``MultimodalBertClf`` keys (src/mmbt.py:237-262).
mmbt_ref.py       fp32 functional restatement of src/mmbt.py (+ the third-party
                  ResNet-152 / pytorch_pretrained_bert 0.6.x math it calls).
bertadam_ref.py   restatement of pytorch_pretrained_bert 0.6.x BertAdam
                  (constructed at train.py:142-147).  No copy of BertAdam is on
                  disk, so this restatement is "parity unpinned" beyond the
                  published formula.
uncertainty_ref.py  member/pass softmax-mean, NLL, ECE (north-star metrics;
                  ECE is build-defined, "parity unpinned").
gen_golden.py     runs the REFERENCE's own src/mmbt.py + src/framework.py
                  (importable here with third-party stubs) to write the golden
                  fixtures under tests/golden/ that pin this restatement.

Pinning status: logits / pooled / embeddings / loss of every forward variant
are pinned against the reference src/mmbt.py running on transformers' BERT
(an independent implementation of the pytorch_pretrained_bert math).  The
ResNet-152 trunk has no third-party implementation in this image
(torchvision is absent): it is pinned only structurally (key names/shapes)
-- "parity unpinned" for its arithmetic.
"""
