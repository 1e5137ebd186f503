"""Minimal gin-config front-end (gin-config is not installed here).

The reference keeps gin files (configs/*.gin) but binds them to nothing
(SURVEY §0).  Here a `.gin` file / `--gin_param` string of `Scope.param = value`
bindings is parsed (comments, Python-literal values, `@name` references kept as
strings, multi-line [...] / (...) values) and the bindings whose scope targets the
entry point (`train.`, `eval_.`, `training_loop.`, `evalution_loop.`, or no scope)
are mapped onto the argparse namespace, so `train.lr=5e-5` == `--lr 5e-5`.
"""
import ast
import re

ENTRY_SCOPES = {"train", "eval_", "eval", "training_loop", "evalution_loop", "eval_robustness"}
_LINE = re.compile(r"^\s*([A-Za-z_][\w.]*)\s*=\s*(.+?)\s*$", re.S)


def _value(text):
    t = text.strip()
    if t.startswith("@"):
        return t
    try:
        return ast.literal_eval(t)
    except (ValueError, SyntaxError):
        return t


def parse_bindings(text):
    """'A.b = 1\\nc=[1,\\n 2]  # x' -> {'A.b': 1, 'c': [1, 2]}"""
    out, buf, depth = {}, "", 0
    for raw in text.splitlines():
        line = raw.split("#", 1)[0]
        if not line.strip() and depth == 0:
            continue
        buf += line + "\n"
        depth += sum(line.count(c) for c in "([{") - sum(line.count(c) for c in ")]}")
        if depth > 0:
            continue
        m = _LINE.match(buf.strip())
        if not m:
            raise ValueError(f"gin: cannot parse binding {buf.strip()!r}")
        out[m.group(1)] = _value(m.group(2))
        buf = ""
    if buf.strip():
        raise ValueError(f"gin: unterminated binding {buf.strip()!r}")
    return out


def apply_to_args(args, bindings, scopes=ENTRY_SCOPES):
    """Set args.<param> for bindings scoped to the entry point; return the unused ones."""
    unused = {}
    for key, val in bindings.items():
        scope, _, name = key.rpartition(".")
        if (scope == "" or scope in scopes) and hasattr(args, name):
            cur = getattr(args, name)
            if isinstance(cur, bool) and not isinstance(val, bool):
                val = bool(val)
            elif isinstance(cur, (int, float)) and not isinstance(cur, bool) and isinstance(val, (int, float)):
                val = type(cur)(val)
            setattr(args, name, val)
        else:
            unused[key] = val
    return unused


def load(args, files=(), params=()):
    text = ""
    for f in files or ():
        with open(f) as fh:
            text += fh.read() + "\n"
    text += "\n".join(params or ())
    return apply_to_args(args, parse_bindings(text)) if text.strip() else {}
