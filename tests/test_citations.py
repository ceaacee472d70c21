"""Audit trail of the restatement: every `src/<file>:<lines>` citation in the repository's code
and docs must point inside the reference file it names, and when the citation names a reference
symbol (`Triangle::bvhIntersect (src/Shape.cpp:297-345)`, `/* PointLight::BasicShading
Light.cpp:238-250 */`, `// ComputeBoundingBox BVH.cpp:268-283`) that symbol must appear in the
cited lines.  A bare `:a-b` continues the file named last before it in the same source file.

Runs only where the reference checkout exists (this container); the GPU box has none."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
FILES = (r"(?:BVH|Scene|Shape|Helper|Light|Camera|Texture|Perlin|Ray|Image|Parser|defs|Material|Instance|"
         r"Transformation|BTNode|main|tinyexr|tinyxml2|happly)\.(?:cpp|h)")
CITE = re.compile(r"(?:src/)?(" + FILES + r")?:(\d+(?:-\d+)?(?:,\s*\d+(?:-\d+)?)*)")
SKIP_DIRS = {".git", "gpurun_out", "profiles", "__pycache__", "build", ".pytest_cache", ".hypothesis"}
# documents written by others (the survey, the judge's review) are not this repository's claims
SKIP_FILES = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "PAPERS.md", "SNIPPETS.md", "test_citations.py"}

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent (GPU box)")


def _ref_lines(name, cache={}):
    if name not in cache:
        with open(os.path.join(REF, name), errors="replace") as f:
            cache[name] = f.read().split("\n")
    return cache[name]


def _ref_symbols(cache={}):
    """Names of the functions the reference defines (a definition line: a name, a parameter list
    and no `;`), minus class names (constructors are matched only when written `Class::Class`)."""
    if not cache:
        defs, classes = set(), set()
        for f in os.listdir(REF):
            if not f.endswith((".cpp", ".h")) or f.startswith(("tinyexr", "tinyxml2", "happly")):
                continue
            for line in _ref_lines(f):
                m = re.match(r"^\s*(?:[\w:<>\*&]+\s+)*?(?:\w+::)?([A-Za-z_]\w*)\s*\([^;]*$", line)
                if m and not re.match(r"^\s*(if|for|while|switch|return|else)\b", line):
                    defs.add(m.group(1))
                classes |= set(re.findall(r"(?:class|struct)\s+([A-Za-z_]\w*)", line))
        cache["defs"], cache["classes"] = defs, classes
    return cache["defs"], cache["classes"]


def _ranges(spec):
    out = []
    for part in spec.split(","):
        a, _, b = part.strip().partition("-")
        out.append((int(a), int(b or a)))
    return out


def citations():
    found = []
    for d, ds, fs in os.walk(ROOT):
        ds[:] = [x for x in ds if x not in SKIP_DIRS]
        for fname in fs:
            if fname in SKIP_FILES or not fname.endswith((".c", ".h", ".cpp", ".hip", ".py", ".md", ".hpp", ".sh")):
                continue
            path = os.path.join(d, fname)
            last = None
            for ln, line in enumerate(open(path, errors="replace"), 1):
                for m in CITE.finditer(line):
                    f, spec = m.group(1), m.group(2)
                    s = m.start()
                    if f:
                        last = f
                    else:
                        if s == 0 or line[s - 1] not in " (," or last is None:
                            continue
                        if m.end() < len(line) and line[m.end()] == "]":     # a Python slice
                            continue
                        f = last
                    found.append((os.path.relpath(path, ROOT), ln, f, spec, line[:s]))
    return found


CITATIONS = citations() if os.path.isdir(REF) else []


def test_there_are_citations():
    assert len(CITATIONS) > 150


@pytest.mark.parametrize("where,ln,ref,spec,before", CITATIONS,
                         ids=[f"{w}:{n}->{f}:{s}" for w, n, f, s, _ in CITATIONS])
def test_citation_resolves(where, ln, ref, spec, before):
    assert os.path.exists(os.path.join(REF, ref)), f"{where}:{ln}: no reference file {ref}"
    lines = _ref_lines(ref)
    n = len(lines) - (1 if lines and lines[-1] == "" else 0)
    rs = _ranges(spec)
    for a, b in rs:
        assert 1 <= a <= b <= n, f"{where}:{ln}: {ref}:{a}-{b} outside the file ({n} lines)"
    # the nearest reference function named before the citation, after any earlier citation on the
    # line (within 60 characters)
    tail = re.split(CITE, before)[-1][-60:] if CITE.search(before) else before[-60:]
    defs, classes = _ref_symbols()
    cand = []
    for tok in re.findall(r"[A-Za-z_~]\w*(?:::[A-Za-z_~]\w*)?", tail):
        cls, _, name = tok.rpartition("::")
        if name in defs and (name not in classes or cls == name) and len(name) > 3:
            cand.append(name)
    if not cand:
        return
    sym = cand[-1]
    body = "\n".join("\n".join(lines[a - 1:b]) for a, b in rs)
    assert re.search(r"\b" + re.escape(sym) + r"\b", body), \
        f"{where}:{ln}: `{sym}` does not appear in {ref}:{spec}"
