"""Options-database semantics (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates
* the options-file loader of the reference ``lib/Parser.py:61-73``: a line is
  stripped, skipped if it contains ``#`` anywhere or is empty, split on single
  spaces, ``key = split[0]``, ``value = split[-1]``; a lone token is a flag;
  keys keep their leading ``-`` (PETSc strips it on insertion);
* the precedence of ``setFromOptions``: an options-DB value wins over the
  programmatic ``setType``/``setTolerances`` (reference ``lib/Solver.py:96-101``,
  ``lib/Preconditioner.py:94-100``).
"""
from __future__ import annotations


def parse_options_lines(lines):
    db = {}
    for _line in lines:
        line = _line.rstrip().lstrip()
        if "#" in line or len(line) == 0:
            continue
        split = line.split(" ")
        if len(split) > 1:
            key, val = split[0], split[-1]
        else:
            key, val = line, None
        db[key.lstrip("-")] = val
    return db


def parse_options_file(path):
    with open(path, "r") as fh:
        return parse_options_lines(fh.readlines())


_TRUE = {None, "", "1", "true", "yes", "on", "TRUE", "True"}


def get(db, prefix, key, default=None, kind=str):
    full = prefix + key
    if full not in db:
        return default
    v = db[full]
    if kind is bool:
        return v in _TRUE
    if v is None:
        return default
    return kind(v)
