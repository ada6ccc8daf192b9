"""Pattern containment helper used by the CLI's --super_pattern filter.

Only the parts of the reference's ``kmerpapa.papa.Pattern`` (src/kmerpapa/papa.py:3-50)
that sit on the path are provided; ``PatternPartition`` is unused by the reference CLI
(its call is commented out at cli.py:286) and is out of scope.
"""
from .pattern_utils import code, matches, set_code, set_perm_code, inv_code


class Pattern:
    """An IUPAC pattern that answers ``kmer in pattern``."""

    def __init__(self, pattern_string):
        self.pattern = pattern_string

    def __contains__(self, context):
        return all(c in set_code[p] for p, c in zip(self.pattern, context))

    def __str__(self):
        return self.pattern

    __repr__ = __str__

    def __len__(self):
        return len(self.pattern)

    def __iter__(self):
        return matches(self.pattern)

    def __and__(self, other):
        out = []
        for a, b in zip(self.pattern, other.pattern):
            both = set_code[a] & set_code[b]
            if not both:
                return None
            out.append(inv_code[both])
        return Pattern("".join(out))

    def __le__(self, other):
        return all(x in set_perm_code[y] for x, y in zip(self.pattern, other.pattern))

    def cardinality(self):
        n = 1
        for x in self.pattern:
            n *= len(code[x])
        return n
