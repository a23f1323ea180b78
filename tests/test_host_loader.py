"""CPU tests of the host-side loader logic that feeds the kernels (no GPU): the corpus-CSV columns
reproduce the reference's RQ4 grouping once the eligible set is applied, and the dictionary
encodings (group key, canonical revisions) behave like the reference's string operations."""
import numpy as np
import pytest

import goldens
from oracle import rq_oracle as orc
from tse_amd.rq import common


@pytest.mark.parametrize("case", goldens.CASES)
@pytest.mark.parametrize("missing_to_g1", [True, False])
def test_corpus_columns_match_grouping(case, missing_to_g1):
    t = goldens.tables(case)
    elig = orc.eligible_projects(t)
    ref_groups, ref_us = common.corpus_groups(t, elig, add_missing_to_g1=missing_to_g1)
    member, corpus_us, order = common.corpus_columns(t)
    is_elig = np.zeros(len(t.projects), bool)
    is_elig[elig] = True
    m = np.where(is_elig, member & 0xF, 0)
    if missing_to_g1:
        m = m | np.where(is_elig & ((member & 0x10) != 0), 1, 0)
    for k in range(4):
        assert np.nonzero(m & (1 << k))[0].tolist() == ref_groups[f"group{k + 1}"]
    for p, us in ref_us.items():
        assert corpus_us[p] == us
    ref_order = common.corpus_order(t, elig)
    assert [p for p in order.tolist() if is_elig[p]] == ref_order


def test_group_key_and_canon():
    t = goldens.tables("tiny")
    gk = t.group_key()
    b = np.nonzero(t.b_modules >= 0)[0][:200]
    text = [str(t.modules_pool[t.b_modules[i]]) + "_" + str(t.revisions_pool[t.b_revisions[i]]) for i in b]
    for i in range(len(b)):
        for j in range(i + 1, min(len(b), i + 20)):
            assert (gk[b[i]] == gk[b[j]]) == (text[i] == text[j])
    canon = t.rev_canon()
    for i in range(len(b) - 1):
        a = sorted(t.revisions_pool[t.b_revisions[b[i]]][1:-2].split(","))
        c = sorted(t.revisions_pool[t.b_revisions[b[i + 1]]][1:-2].split(","))
        assert (canon[b[i]] == canon[b[i + 1]]) == (a == c)
