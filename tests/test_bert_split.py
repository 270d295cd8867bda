"""Where the frozen encoder splits a batch into a whole-wave chunk and a tail chunk
(irc_amd.bert.BertModel._split_point; host logic, no GPU)."""
import dataclasses


def test_split_point():
    from irc_amd.bert import BERT_BASE, BertModel

    m = BertModel(dataclasses.replace(BERT_BASE, num_hidden_layers=1), seed=0)
    assert m._split_point(512, 64) == 0      # exactly 32768 rows: whole waves already
    assert m._split_point(512, 60) == 0      # below one set of waves
    assert m._split_point(512, 65) == 504    # 32760 + 520 rows
    assert m._split_point(512, 72) == 455
    assert m._split_point(512, 80) == 409    # remainder 8192 rows = 1/4: still split
    assert m._split_point(512, 81) == 0      # remainder above 1/4
    assert m._split_point(1024, 64) == 0     # 65536 rows: two whole sets
    assert m._split_point(1024, 66) == 992   # 67584 rows: 65472 + 2112
    m.split_tail = False
    assert m._split_point(512, 65) == 0
