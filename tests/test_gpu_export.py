"""GPU: N4 export contract -- the named outputs and sub_models of AutoInt and the staytime model
(autoint:53-54, staytime/VideoDnn.py:193-215) equal the models' own outputs, and a checkpoint
taken mid-training resumes to the same trajectory (config 5 at 20k rows, deterministic push)."""
import numpy as np
import pytest
import torch

from recommendsystem_amd import export

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_autoint_named_output_and_sub_model():
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig
    cfg = AutoIntConfig(vocab_per_field=100)
    m = AutoInt(cfg, device=DEV, seed=3, max_batch=64)
    ids = torch.randint(0, 1000, (64, cfg.num_fields), device=DEV)
    with torch.no_grad():
        p = m(ids)
        out = export.autoint_predict(m, ids)
        assert list(out) == ["video_id_rank_skip_model"]
        assert torch.equal(out["video_id_rank_skip_model"], p)
        sub = export.autoint_sub_model(m)(m.embedding(ids))
        assert torch.equal(sub["video_id_rank_skip_model"], p)


def test_staytime_sub_models():
    from recommendsystem_amd.workloads import StaytimeRoughRank, staytime_batch
    j = StaytimeRoughRank(rows=20_000, device=DEV, seed=2)
    rng = np.random.default_rng(1)
    st_ids, seq_ids, seq_offs = staytime_batch(rng, 32, j, DEV)[:3]
    with torch.no_grad():
        emb = j.fields(st_ids)
        seqs, masks = zip(*[j.seqs[s](seq_ids[s], seq_offs[s]) for s in range(j.st_cfg.num_seq)])
        subs = export.staytime_sub_models(j.staytime)
        tr = subs["sub_model_train"](emb, list(seqs), list(masks))
        pr = subs["sub_model_predict"](emb, list(seqs), list(masks))
    names = list(export.STAYTIME_TASKS)
    assert list(tr) == names and list(pr) == names
    stay = tr[names[0]]
    assert stay.shape == (32, 401) and pr[names[0]].shape == (32, 1)
    assert torch.equal(pr[names[0]], stay[:, 400:401])
    torch.testing.assert_close(stay[:, :400].sum(1), torch.ones(32, device=DEV), rtol=0, atol=1e-5)
    assert bool((pr[names[0]] >= 0).all())
    for k in names[1:]:
        assert torch.equal(tr[k], pr[k])
    assert export.staytime_tensor_names("train")[names[0]] == names[0] + "_l"


def _trainer(seed):
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd.workloads import StaytimeRoughRank
    j = StaytimeRoughRank(rows=20_000, device=DEV, seed=seed)
    j.table.deterministic = True
    # the DSSM at its own lr (rough_rank/model.py:209): a second dense segment with its own Adam
    # step counter, which a resume must restore too
    return j, Trainer(j, 5e-4, [j.table], lr_groups=[(j.dssm, j.rr_cfg.lr_dense)])


def test_checkpoint_resume_matches_uninterrupted(tmp_path):
    from recommendsystem_amd.workloads import staytime_batch
    a, ta = _trainer(4)
    rng = np.random.default_rng(2)
    batches = [staytime_batch(rng, 64, a, DEV) for _ in range(3)]
    la = [float(ta.step(*b)) for b in batches]
    b, tb = _trainer(4)
    for bt in batches[:2]:
        tb.step(*bt)
    torch.cuda.synchronize()
    export.save_checkpoint(str(tmp_path), b, tb)
    c, tc = _trainer(99)
    export.load_checkpoint(str(tmp_path), c, tc)
    assert int(tc.step_count) == 2
    assert all(int(cnt) == 2 for *_, cnt in tc.segments) and len(tc.segments) > 1
    lc = float(tc.step(*batches[2]))
    np.testing.assert_allclose(lc, la[2], rtol=1e-6)
    torch.cuda.synchronize()
    torch.testing.assert_close(c.table.weight, a.table.weight, rtol=1e-5, atol=1e-6)
    for p, q in zip(c.parameters(), a.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-6)
