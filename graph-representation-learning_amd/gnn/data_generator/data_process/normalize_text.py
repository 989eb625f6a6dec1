"""Text normalisation applied before the bag-of-characters encoding.

Restates the reference's rule set (gnn/data_generator/data_process/utils/
normalize_text.py): lower-case, NFKC, then in order: ASCII digits -> "0",
"'" -> '"', ";" -> ",", "_" -> "-", tab/newline/CR -> " ", Unicode dashes (Pd)
-> "-", Unicode spaces (Zs/Zl/Zp) -> " ", dot/stop punctuation (Po whose name
has "DOT"/"STOP" as a word part) -> ".", opening brackets -> "(", closing
brackets -> ")".  Brackets are the Ps/Pe/Pi/Pf characters, mirrored ones first
then the rest, each in code-point order, paired (opening, closing) two by two
-- the reference's pairing, reproduced exactly.
"""
from __future__ import annotations

import functools
import sys
import unicodedata
from typing import Dict, List, Optional


def _scan(pred) -> str:
    mirrored, other = [], []
    for cp in range(sys.maxunicode + 1):
        c = chr(cp)
        if pred(c):
            (mirrored if unicodedata.mirrored(c) else other).append(c)
    return "".join(mirrored) + "".join(other)


def _dot_name(c: str) -> bool:
    if unicodedata.category(c) != "Po":
        return False
    name = unicodedata.name(c, None)
    if name is None:
        return False
    parts = ("DOT ", " DOT", " STOP", "STOP ")
    return name in parts or any(p in name for p in parts)


@functools.lru_cache(maxsize=1)
def _steps() -> List[Dict[int, str]]:
    brackets = _scan(lambda c: unicodedata.category(c) in ("Ps", "Pe", "Pi", "Pf"))
    lefts, rights = brackets[0::2], brackets[1::2]
    dashes = _scan(lambda c: unicodedata.category(c) == "Pd")
    spaces = _scan(lambda c: unicodedata.category(c) in ("Zs", "Zl", "Zp"))
    dots = _scan(_dot_name)

    def table(chars: str, to: str) -> Dict[int, str]:
        return {ord(c): to for c in chars}

    return [table("0123456789", "0"), table("'", '"'), table(";", ","), table("_", "-"), table("\t\n\r", " "),
            table(dashes, "-"), table(spaces, " "), table(dots, "."), table(lefts, "("), table(rights, ")")]


def normalize_text(text: str, corpus: Optional[List[str]] = None) -> str:
    text = unicodedata.normalize("NFKC", text.lower())
    for step in _steps():
        text = text.translate(step)
    if corpus is not None:
        text = "".join(c if c in corpus else "�" for c in text)
    return text
