"""A process-global options database standing in for ``PETSc.Options()``.

The reference fills PETSc's options DB from a file (lib/Parser.py:61-73) and
every KSP/PC reads it in ``setFromOptions``.  Here the same key/value pairs are
kept in ``DB`` and forwarded to libpls.so, which applies them with the same
prefix rules and precedence.
"""
DB = {}


class Options:
    def setValue(self, key, value):
        DB[str(key).lstrip("-")] = None if value is None else str(value)

    def getValue(self, key):
        return DB.get(str(key).lstrip("-"))

    def delValue(self, key):
        DB.pop(str(key).lstrip("-"), None)

    def getAll(self):
        return dict(DB)

    def clear(self):
        DB.clear()


def to_text(extra=None):
    lines = []
    merged = dict(DB)
    if extra:
        merged.update(extra)
    for k, v in merged.items():
        lines.append(k if v is None else f"{k} {v}")
    return "\n".join(lines)
