"""BERT model: padding semantics + HF state-dict interop on CPU; HIP path vs fp32 CPU
reference on the GPU (K2 non-causal flash attention with key-padding lengths, BDA-LN,
bias-GeLU)."""
import copy

import pytest
import torch

from mxtrain.models.bert import BERT_CONFIGS, BertConfig, BertForSequenceClassification


def _tiny(**kw):
    return BertConfig(**dict(BERT_CONFIGS["bert-tiny"], **kw))


def test_padding_does_not_change_logits():
    torch.manual_seed(0)
    m = BertForSequenceClassification(_tiny(hidden_dropout_prob=0.0)).eval()
    ids = torch.randint(5, 1000, (1, 13))
    full = m(ids)["logits"]
    pad = torch.zeros(1, 32, dtype=torch.long)
    pad[0, :13] = ids
    am = torch.zeros(1, 32, dtype=torch.long)
    am[0, :13] = 1
    torch.testing.assert_close(m(pad, attention_mask=am)["logits"], full, rtol=1e-4, atol=1e-5)


def test_hf_state_dict_roundtrip_and_backward():
    m = BertForSequenceClassification(_tiny())
    sd = m.hf_state_dict()
    assert "bert.encoder.layer.1.attention.self.value.weight" in sd
    m2 = BertForSequenceClassification(_tiny(), seed=7)
    m2.load_hf_state_dict(sd)
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(a, b, msg=n)
    ids = torch.randint(5, 1000, (4, 24))
    out = m(ids, labels=torch.tensor([0, 1, 1, 0]))
    out["loss"].backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.gpu
def test_bert_gpu_matches_cpu_reference():
    torch.manual_seed(0)
    cfg = BertConfig(**dict(BERT_CONFIGS["bert-tiny"], hidden_size=256, num_attention_heads=4, intermediate_size=1024,
                            hidden_dropout_prob=0.0))
    cpu = BertForSequenceClassification(cfg).train()
    gpu = copy.deepcopy(cpu).cuda().train()
    B, S = 4, 128
    ids = torch.randint(5, 1000, (B, S))
    am = torch.ones(B, S, dtype=torch.long)
    for b, L in enumerate((128, 77, 5, 64)):
        am[b, L:] = 0
        ids[b, L:] = 0
    labels = torch.tensor([0, 1, 1, 0])
    oc = cpu(ids, attention_mask=am, labels=labels)
    og = gpu(ids.cuda(), attention_mask=am.cuda(), labels=labels.cuda())
    torch.testing.assert_close(og["logits"].cpu(), oc["logits"], rtol=5e-2, atol=5e-2)
    oc["loss"].backward()
    og["loss"].backward()
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        gc, gg = pc.grad, pg.grad.cpu()
        err = (gg - gc).norm() / (gc.norm() + 1e-6)
        assert err < 0.1, (n, float(err))
