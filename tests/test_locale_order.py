"""localeCompare parity (RiskAnalyzer.ts:57-60 sorts service names with it):
the product's collation key (kmamiz_amd/risk.py) and the oracle's against the
order the reference's Node (12.22.9, ICU 70.1) produced for a corpus of
service names (tests/golden/locale_order.json, tests/golden/gen_locale_order.js)."""
import functools
import json
import os

from kmamiz_amd.risk import _MARK_RANK, _PUNCT, _collation_key
from oracle.kmz_oracle import _locale_key

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "locale_order.json")))


def _cmp(key):
    def c(a, b):
        ka, kb = key(a), key(b)
        return (ka > kb) - (ka < kb)
    return c


def test_product_key_sorts_like_node():
    assert sorted(GOLD["corpus"], key=_collation_key) == GOLD["sorted"]


def test_product_key_signs_like_node():
    c = _cmp(_collation_key)
    s = GOLD["sorted"]
    assert [c(s[i - 1], s[i]) for i in range(1, len(s))] == GOLD["signs"]


def test_oracle_key_sorts_like_node():
    assert sorted(GOLD["corpus"], key=_locale_key) == GOLD["sorted"]
    c = _cmp(_locale_key)
    s = GOLD["sorted"]
    assert [c(s[i - 1], s[i]) for i in range(1, len(s))] == GOLD["signs"]


def test_product_tables_match_node():
    ign = set(GOLD["punct_ignorable"])
    assert "".join(c for c in GOLD["punct_sorted"] if c not in ign) == _PUNCT
    ranks = [_MARK_RANK[m] for m in GOLD["marks_sorted"]]
    # localeCompare(previous, next): -1 while the rank rises, 0 on a tie
    assert [(a > b) - (a < b) for a, b in zip(ranks, ranks[1:])] == GOLD["marks_signs"]
