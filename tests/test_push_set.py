"""What travels to the GPU box.

gpurun ships this tree minus .git/, gpurun_out/, Python caches and the paths .gpurunignore lists (tar exclude
patterns).  Nothing derived from the reference's Python may travel: no shipped source file names the reference
checkout outside comments or docstrings, so every script that imports it (the golden generators, the
reference-loop study) must be listed in .gpurunignore.  The shipped tests that need the G9 batches import
tests/golden/g9_batches.py, which is plain data generation."""
import ast
import fnmatch
import io
import os
import re
import tokenize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NEEDLE = "/root/" + "reference"
CODE_EXT = {".py", ".sh", ".c", ".h", ".cpp", ".hip", ".inc", ".cc"}


def _patterns():
    pats = []
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        for ln in f:
            ln = ln.strip()
            if ln and not ln.startswith("#"):
                pats.append(ln)
    return pats


def _excluded(rel, pats):
    """tar --exclude semantics for the patterns used here: './x' anchors at the top, a bare pattern matches any
    path component suffix; wildcards match '/'."""
    dotted = "./" + rel
    parts = rel.split("/")
    for p in pats:
        if p.startswith("./"):
            if fnmatch.fnmatchcase(dotted, p) or any(fnmatch.fnmatchcase("./" + "/".join(parts[:i]), p)
                                                     for i in range(1, len(parts))):
                return True
        elif any(fnmatch.fnmatchcase("/".join(parts[i:]), p) for i in range(len(parts))) or \
                any(fnmatch.fnmatchcase(c, p) for c in parts):
            return True
    return False


def shipped_files():
    pats = _patterns()
    out = []
    for d, dirs, files in os.walk(ROOT):
        rel_d = os.path.relpath(d, ROOT)
        dirs[:] = [x for x in dirs if x not in (".git", "gpurun_out", "__pycache__", ".pytest_cache")
                   and not _excluded(os.path.normpath(os.path.join(rel_d, x)), pats)]
        for fn in files:
            rel = os.path.normpath(os.path.join(rel_d, fn))
            if not _excluded(rel, pats) and not fn.endswith(".pyc"):
                out.append(rel)
    return out


def _python_code_text(src):
    """The source with comments and docstrings removed (strings that are not docstrings kept)."""
    tree = ast.parse(src)
    doc_lines = set()
    for node in ast.walk(tree):
        if isinstance(node, (ast.Module, ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            body = node.body
            if body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant) \
                    and isinstance(body[0].value.value, str):
                doc_lines.add((body[0].lineno, body[0].col_offset))
    kept = []
    for tok in tokenize.generate_tokens(io.StringIO(src).readline):
        if tok.type == tokenize.COMMENT:
            continue
        if tok.type == tokenize.STRING and tok.start in doc_lines:
            continue
        kept.append(tok.string)
    return " ".join(kept)


def _c_code_text(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def _sh_code_text(src):
    return "\n".join(re.sub(r"(^|\s)#.*$", " ", ln) for ln in src.splitlines())


def test_build_only_reference_scripts_are_not_shipped():
    ship = set(shipped_files())
    for rel in ("scripts/reference_loop_study.py", "scripts/stage1_strong_replay.py", "tests/golden/make_golden.py",
                "tests/golden/make_td3_golden.py", "tests/golden/extract_stage3_actor.py",
                "tests/golden/extract_checkpoint_actors.py", "tests/golden/extract_resume_checkpoint.py"):
        assert os.path.exists(os.path.join(ROOT, rel)), rel
        assert rel not in ship, f"{rel} would travel to the GPU box"
    # what the GPU run needs still travels
    for rel in ("bench.py", "__graft_entry__.py", "tests/golden/g9_batches.py", "tests/test_gpu_learner.py",
                "include/hockey.h", "oracle/hk_oracle.c"):
        assert rel in ship, rel


def test_no_shipped_code_names_the_reference_checkout():
    bad = []
    for rel in shipped_files():
        ext = os.path.splitext(rel)[1]
        if ext not in CODE_EXT and os.path.basename(rel) != "Makefile":
            continue
        try:
            src = open(os.path.join(ROOT, rel), encoding="utf-8").read()
        except (UnicodeDecodeError, OSError):
            continue
        if NEEDLE not in src:
            continue
        if ext == ".py":
            code = _python_code_text(src)
        elif ext == ".sh" or os.path.basename(rel) == "Makefile":
            code = _sh_code_text(src)
        else:
            code = _c_code_text(src)
        if NEEDLE in code:
            bad.append(rel)
    assert not bad, f"shipped files naming the reference outside comments/docstrings: {bad}"
