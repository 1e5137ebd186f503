"""HIP-graph replay of the whole MMBT training step (src/graphs.py; bench.py --graph).

* The dropout seed counter (include/mmu.h mmu_set_seed_offset): a counter of 0 leaves every
  dropout launch as eager execution draws it (same loss and gradients as no counter), a
  counter of 1 draws other masks.
* Replay == eager: a graph-replayed training step (forward with attention / hidden / embedding
  dropout, backward with the deferred side-stream weight gradients, fused BertAdam) equals the
  eager step run with the same host-drawn seeds and the same counter value, step after step
  (loss to 1e-5; the parameters after 4 optimizer steps to 1e-4 of their update, without the
  attention key biases, whose zero gradient BertAdam turns into sign-of-noise steps; on the
  full model, whose float-atomic gradient sums differ from run to run, within 3x of the eager
  step's own run-to-run spread, measured in the test);
  consecutive replays draw new masks.
Model: the small MMBT (2 BERT layers, one Bottleneck per stage), batch 8, in training mode
(batch-statistic BatchNorm), the reference's step (src/framework.py:276-304)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B, T, P = 8, 16, 0.1


def _model(sd=None, full=False):
    from oracle.weights import FULL_C, SMALL, make_state_dict
    from src.mmbt import MultimodalBertClf
    from src.optim import BertAdam
    from src.testing import make_args, small_args
    torch.manual_seed(0)
    mk = make_args if full else small_args
    m = MultimodalBertClf(mk(bert_hidden_dropout=P, bert_attn_dropout=P, dropout=P))
    m.load_state_dict(sd if sd is not None else make_state_dict(0, FULL_C if full else SMALL), strict=True)
    m = m.to("cuda:0").train()
    named = list(m.named_parameters())
    nd = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
    groups = [{"params": [p for n, p in named if not any(k in n for k in nd)], "weight_decay": 0.01},
              {"params": [p for n, p in named if any(k in n for k in nd)], "weight_decay": 0.0}]
    return m, BertAdam(groups, lr=1e-5, warmup=0.1, t_total=20.0)


def _batch(full=False):
    from oracle.weights import SMALL
    from src.testing import synthetic_batch
    if full:  # BASELINE config 4's per-rank shapes at a small batch: L = 513
        x, y = synthetic_batch(4, 508, lens=[508, 300, 508, 77], seed=4)
    else:
        x, y = synthetic_batch(B, T, vocab=SMALL.vocab, lens=[16, 9, 16, 12, 5, 16, 14, 16], seed=4)
    return tuple(t.to("cuda:0") for t in x), y.to("cuda:0")


def _stepper(m, o, x, y, optimize=True):
    def step():
        o.zero_grad()
        loss = m.compute_loss(m(*x), y)
        loss.backward()
        if optimize:
            o.step()
        return loss
    return step


def test_seed_counter_zero_is_the_eager_draw(dev):
    from src import kernels as K
    torch.backends.cudnn.deterministic = True
    m, o = _model()
    x, y = _batch()
    step = _stepper(m, o, x, y, optimize=False)
    out = []
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    try:
        for value in (None, None, 0, 1):  # (the first step builds the lazily made buffers)
            if value is not None:
                ctr.fill_(value)
            K.set_seed_offset(None if value is None else ctr)
            torch.manual_seed(11)  # the host-drawn seeds (src/mmbt.py _seed)
            loss = step()
            torch.cuda.synchronize()
            out.append((loss.item(), m.store.grad.clone()))
    finally:
        K.set_seed_offset(None)
    (lw, gw), (l0, g0), (l1, g1), (l2, g2) = out
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    print(f"\n[seed counter] loss first {lw:.6f} (grad rel diff {rel(gw, g0):.2e}) none {l0:.6f} / zero {l1:.6f} / "
          f"one {l2:.6f}; grad rel diff zero {rel(g1, g0):.2e}, one {rel(g2, g0):.2e}")
    noise = rel(gw, g0)  # the eager step against itself (float-atomic summation order)
    assert abs(l1 - l0) <= max(3 * abs(lw - l0), 1e-7 * abs(l0)) and rel(g1, g0) <= max(3 * noise, 1e-6)
    assert rel(g2, g0) > max(30 * noise, 1e-2)


@pytest.mark.parametrize("full", [False, True])
def test_graph_replay_equals_eager_steps(dev, full):
    """full: ResNet-152 + 12 BERT layers at L = 513, batch 4 (MIOpen convs, the side stream's
    deferred weight gradients and the trunk's residual-stream residue inside the capture)."""
    from src import kernels as K
    torch.backends.cudnn.deterministic = True
    from src.graphs import StepGraph
    x, y = _batch(full)
    ma, oa = _model(full=full)
    sd0 = {k: v.detach().cpu().clone() for k, v in ma.state_dict().items()}
    torch.manual_seed(21)
    g = StepGraph(_stepper(ma, oa, x, y), dev, warmup=1)
    # host RNG state after the capture's draws (the graph's seeds): the eager arm restores the
    # state from before the capture for each of its steps instead
    losses_a = []
    for _ in range(3):
        losses_a.append(g.replay().item())
    torch.cuda.synchronize()
    flat_a = ma.store.flat.clone()
    ctr_a = int(g.counter.item())
    g.release()
    del g

    def eager():
        """the eager arm: the StepGraph's warm-up step, then 3 steps with the capture's host
        seeds and the counter values the replays ran with"""
        mb, ob = _model(sd0, full=full)
        flat0 = mb.store.flat.clone()
        step_b = _stepper(mb, ob, x, y)
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        K.set_seed_offset(ctr)
        try:
            torch.manual_seed(21)
            ctr.fill_(1)
            step_b()  # = StepGraph's eager warmup step (counter 1)
            rng = torch.get_rng_state()  # the capture drew its seeds from here
            losses = []
            for k in range(3):
                torch.set_rng_state(rng)
                ctr.fill_(2 + k)  # the replay's first node advanced the counter to 2, 3, 4
                losses.append(step_b().item())
            torch.cuda.synchronize()
        finally:
            K.set_seed_offset(None)
        # without the key biases: their true gradient is 0 (softmax shift invariance), so BertAdam
        # moves them by the sign of float-atomic noise
        keep = torch.ones_like(flat0, dtype=torch.bool)
        for n in mb.store.names:
            if n.endswith("attention.self.key.bias"):
                keep[mb.store.offsets[n]:mb.store.offsets[n] + mb.store.params[n].numel()] = False
        out = (losses, mb.store.flat.clone(), flat0, keep)
        del mb, ob
        torch.cuda.empty_cache()
        return out

    losses_b, flat_b, flat0, keep = eager()
    rel = lambda u, v: ((u - v)[keep].norm() / (v - flat0)[keep].norm()).item()  # noqa: E731  (of the update)
    d = rel(flat_a, flat_b)
    moved = (flat_b - flat0).norm().item()
    # the floor: the eager step against itself (float-atomic summation order: bias-gradient
    # column sums, embedding-row gradients), which BertAdam amplifies on near-zero gradients
    losses_c, flat_c, _, _ = eager()
    d_ee = rel(flat_c, flat_b)
    l_ee = max(abs(a - b) for a, b in zip(losses_c, losses_b))
    print(f"\n[graph{' full' if full else ''}] replay losses {losses_a}, eager {losses_b}, eager again {losses_c}; "
          f"counter {ctr_a}; params after 4 steps: replay vs eager {d:.2e}, eager vs eager {d_ee:.2e} of the update "
          f"(moved {moved:.3e})")
    assert ctr_a == 4
    if full:
        # the first replay runs on the eager warm-up's parameters: its loss is the eager one (any
        # seed / mask / capture error shows here); later steps carry the float-atomic gradient
        # noise through BertAdam, whose spread is multimodal on the full model (step-2 losses
        # 3.76144 / 3.76147 / 3.76149 across runs of either arm, profiles/r6_graph_floor.txt)
        assert abs(losses_a[0] - losses_b[0]) <= 1e-6 * abs(losses_b[0]), (losses_a, losses_b)
        for a, b in zip(losses_a[1:], losses_b[1:]):
            assert abs(a - b) <= max(1e-3 * abs(b), 3 * l_ee), (losses_a, losses_b, losses_c)
    else:
        for a, b in zip(losses_a, losses_b):
            assert abs(a - b) <= max(1e-5 * abs(b), 3 * l_ee), (losses_a, losses_b, losses_c)
    assert len(set(losses_a)) == 3, "consecutive replays drew the same dropout masks"
    assert moved > 0
    # full model: the eager step's own spread is bimodal -- one float-atomic order flip in the first
    # optimizer steps moves the 4-step update by ~9e-3 or not at all (12 samples, with and without the
    # downsample sink: replay vs eager 4.3e-4 ... 9.1e-3, eager vs eager 1.4e-3 ... 9.0e-3,
    # profiles/r6_graph_floor.txt), so two eager runs can agree while the replay sits in the other
    # mode; the bar is 3x the spread measured here or, on the full model, 2x the largest spread
    # recorded there
    full_floor = 1.8e-2 if full else 0.0
    assert d <= max(1e-4, 3 * d_ee, full_floor), (d, d_ee)
