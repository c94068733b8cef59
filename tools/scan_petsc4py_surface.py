"""AST scan of the reference's petsc4py call surface on the hot path's host
files -> tests/golden/petsc4py_surface.json.

Build-container tool: it parses the reference's Python sources as text (ast,
nothing imported or run) and is not used on the GPU box.  Scope: the files
and line ranges SURVEY 8(b) names for the drop-in --

  src/matrices/mat_fs.py, src/matrices/mat_ns.py, src/solver/kle_solver.py,
  src/cases/base_problem.py:111-222, src/boundaries/boundary_conditions.py:1,191-278

Every call, operator and attribute whose receiver is a petsc4py object is
recorded as (class, member, kind) with its sites and argument shapes.  The
receiver's petsc4py class comes from the imports (`PETSc.Mat()`, names
imported from petsc4py.PETSc) and, for variables and attributes, from the
RECEIVERS table below (what each name holds in those files: read off their
constructors, e.g. mat_fs.py:47 self.K = self.createEmptyMat(...) ->
mat_fs.py:103 PETSc.Mat().createAIJ).  Calls on receivers that are neither
petsc4py objects nor in the IGNORED table (the Domain, loggers, numpy, Python
sets and lists) are listed under "unclassified" so that nothing is dropped
silently; the committed output has none.

  python tools/scan_petsc4py_surface.py [--ref /root/reference] [--out tests/golden/petsc4py_surface.json]
"""
import argparse
import ast
import json
import os
import re
import sys

SCOPE = [
    ("src/matrices/mat_fs.py", None),
    ("src/matrices/mat_ns.py", None),
    ("src/solver/kle_solver.py", None),
    ("src/cases/base_problem.py", [(111, 222)]),
    ("src/boundaries/boundary_conditions.py", [(1, 1), (191, 278)]),
]

# receiver expression (ast.unparse, regex, full match) -> petsc4py class
RECEIVERS = [
    (r"self\.(K|Krhs|Rw|Rd|Rwfs|Rdfs|Kfs|Krhsfs|Curl|SrT|DivSrT)", "Mat"),
    (r"self\.operator\.(Curl|SrT|DivSrT)", "Mat"),
    (r"self\.mat\.(K|Krhs|Rw|Rd|Rwfs|Rdfs|Kfs|Krhsfs)", "Mat"),
    (r"(m|mat|K|Kfs)", "Mat"),                                     # mat_fs.py:17,103; kle_solver.py:14,23
    (r"self\.(weigCurl|weigSrT|weigDivSrT|_VtensV|_Aux1|vort)", "Vec"),
    (r"self\._KleSolver__(vel|velFS)|self\.__(vel|velFS)", "Vec"),
    (r"(vec|vel|vort|rhs|velFS|f|proc)", "Vec"),                   # base_problem.py:111-222, boundary_conditions.py:259
    (r"self\.(solver|solverFS)", "KSP"),                           # kle_solver.py:15,24 KspSolver(KSP)
    (r"pc", "PC"),
    (r"(inds|bcIS)", "IS"),                                        # boundary_conditions.py:187,210
    (r"self\.comm|COMM_WORLD|PETSc\.COMM_WORLD", "Comm"),
    (r"self\.comm\.tompi4py\(\)", "mpi4py.Comm"),
]
# receivers that are not petsc4py objects
IGNORED = [r"self\.dom", r"self\.logger", r"np", r"self\.kle", r"self\.operator", r"self\.viewer", r"self\.ts",
           r"self\.solverKLE", r"self\.mat", r"self", r"super\(\)", r"bc", r"b", r"self\.opts", r"self\.config",
           r"self\.timer\w*", r"logging", r"functionLib", r"initialConditions", r"options", r"indicesVelSet",
           r"globalNormalIndicesNS", r"globalTangIndicesNS", r"normalDofs", r"tangentialDofs", r"indices2one",
           r"indices2onefs", r"inds", r"dofs", r"locDofs", r"locTang", r"locIndices", r"removeSet",
           r"remoteIndices", r"indicesVel", r"importlib", r"self\.__ByType\[bcType\]",
           r"self\._BoundaryConditions__\w+", r"self\.__\w+", r"connectivity", r"connect", r"vel\[tang\]",
           r"bc\.\w+\(.*\)"]
# methods of the ignored Python containers / numpy that share names with nothing petsc4py
PY_METHODS = {"append", "add", "update", "copy", "index", "getLogger", "repeat", "array", "zeros", "arange",
              "tile", "items", "get", "info", "debug", "import_module"}
BUILTIN_OPS = {ast.Mult: "__mul__", ast.Add: "__add__", ast.Sub: "__sub__", ast.Div: "__truediv__"}


def in_scope(line, ranges):
    return ranges is None or any(a <= line <= b for a, b in ranges)


def arg_shape(node):
    """A coarse shape of one argument: literal kinds, containers, tuples."""
    if isinstance(node, ast.Constant):
        return "None" if node.value is None else type(node.value).__name__
    if isinstance(node, (ast.List, ast.ListComp)):
        return "list"
    if isinstance(node, ast.Tuple):
        return "(" + ",".join(arg_shape(e) for e in node.elts) + ")"
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        inner = arg_shape(node.operand)
        return inner if inner in ("int", "float") else "expr"
    if isinstance(node, ast.Call):
        f = ast.unparse(node.func)
        if f in ("list", "set", "range"):
            return f
        if f.startswith("np.") or f == "np.repeat":
            return "ndarray"
        return "call"
    if isinstance(node, ast.Subscript):
        return "subscript"
    if isinstance(node, ast.Name):
        return "name"
    if isinstance(node, ast.Attribute):
        return "attr"
    if isinstance(node, ast.BinOp):
        return "expr"
    return type(node).__name__


class Scan(ast.NodeVisitor):
    def __init__(self, fname, ranges, petsc_names, table):
        self.f, self.ranges, self.petsc_names, self.t = fname, ranges, petsc_names, table
        self.unclassified = []
        self.cls_stack = []
        self.py_locals = [set()]  # per function: names bound to instances of the reference's own classes
        self.sub_methods = set()  # methods the reference defines on its petsc4py subclasses (KspSolver)

    def cls_of(self, node):
        """petsc4py class of the value of expression node, or None."""
        src = ast.unparse(node)
        if isinstance(node, ast.Name) and node.id in self.py_locals[-1]:
            return None  # (e.g. base_problem.py:159 mat = MatFS(): the reference's class, not a Mat)
        # constructors: PETSc.Mat(), Mat() (imported), and their create* chains
        if isinstance(node, ast.Call):
            f = node.func
            if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "PETSc":
                return f.attr
            if isinstance(f, ast.Name) and f.id in self.petsc_names:
                return f.id
            if isinstance(f, ast.Attribute) and f.attr.startswith("create"):
                return self.cls_of(f.value)
            if isinstance(f, ast.Attribute) and f.attr == "tompi4py":
                return "mpi4py.Comm"
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "PETSc":
            return "Comm" if node.attr == "COMM_WORLD" else None
        if isinstance(node, ast.Name) and node.id == "self" and self.cls_stack and self.cls_stack[-1] == "KspSolver":
            return "KSP"  # kle_solver.py:49 class KspSolver(KSP)
        if isinstance(node, ast.BinOp) and type(node.op) in BUILTIN_OPS:
            a = self.cls_of(node.left)
            return a if a in ("Vec", "Mat") and self.cls_of(node.right) != "Vec" else ("Vec" if a else None)
        for pat, c in RECEIVERS:
            if re.fullmatch(pat, src):
                return c
        return None

    def rec(self, cls, member, kind, node, args=(), kws=()):
        key = f"{cls}.{member}"
        e = self.t.setdefault(key, {"class": cls, "member": member, "kind": kind, "sites": [], "forms": []})
        e["sites"].append(f"{self.f}:{node.lineno}")
        form = {"args": [arg_shape(a) for a in args], "kwargs": sorted(k for k in kws if k)}
        if form not in e["forms"]:
            e["forms"].append(form)

    def visit_ClassDef(self, node):
        self.cls_stack.append(node.name)
        for b in node.bases:
            if isinstance(b, ast.Name) and b.id in self.petsc_names:
                self.sub_methods |= {f.name for f in node.body if isinstance(f, ast.FunctionDef)}
                if in_scope(node.lineno, self.ranges):
                    self.rec(b.id, "__subclass__", "subclass", node)
        self.generic_visit(node)
        self.cls_stack.pop()

    def visit_FunctionDef(self, node):
        loc = set()
        for n in ast.walk(node):
            if isinstance(n, ast.Assign) and isinstance(n.value, ast.Call) and isinstance(n.value.func, ast.Name):
                fid = n.value.func.id
                if fid[:1].isupper() and fid not in self.petsc_names:
                    loc |= {t.id for t in n.targets if isinstance(t, ast.Name)}
        self.py_locals.append(loc)
        self.generic_visit(node)
        self.py_locals.pop()

    def visit_Call(self, node):
        if in_scope(node.lineno, self.ranges):
            f = node.func
            kws = [k.arg for k in node.keywords]
            if isinstance(f, (ast.Name, ast.Attribute)) and self.cls_of(f) == "KSP":
                self.rec("KSP", "__call__", "call", node, node.args, kws)  # kle_solver.py:35 self.solver(b, x)
            elif isinstance(f, ast.Attribute):
                rc = self.cls_of(f.value)
                if rc == "KSP" and f.attr in self.sub_methods:
                    pass  # (the subclass's own method, kle_solver.py:54 createSolver)
                elif rc:
                    self.rec(rc, f.attr, "method", node, node.args, kws)
                else:
                    c0 = self.cls_of(node)
                    src = ast.unparse(f.value)
                    if c0 and isinstance(f.value, ast.Name) and f.value.id == "PETSc":
                        self.rec(c0, "__init__", "constructor", node, node.args, kws)
                    elif (not any(re.fullmatch(p, src) for p in IGNORED) and f.attr not in PY_METHODS and
                          src not in self.py_locals[-1]):
                        self.unclassified.append(f"{self.f}:{node.lineno}: {ast.unparse(node)[:100]}")
            elif isinstance(f, ast.Name) and f.id in self.petsc_names:
                self.rec(f.id, "__init__", "constructor", node, node.args, kws)
            else:
                rc = self.cls_of(f)
                if rc == "KSP":
                    self.rec("KSP", "__call__", "call", node, node.args, kws)
        self.generic_visit(node)

    def visit_BinOp(self, node):
        if in_scope(node.lineno, self.ranges) and type(node.op) in BUILTIN_OPS:
            a, b = self.cls_of(node.left), self.cls_of(node.right)
            if a in ("Mat", "Vec"):
                self.rec(a, BUILTIN_OPS[type(node.op)], "operator", node, [node.right])
                e = self.t[f"{a}.{BUILTIN_OPS[type(node.op)]}"]
                e.setdefault("operand_classes", [])
                oc = b or arg_shape(node.right)
                if oc not in e["operand_classes"]:
                    e["operand_classes"].append(oc)
        self.generic_visit(node)

    def visit_AugAssign(self, node):
        if in_scope(node.lineno, self.ranges) and type(node.op) in BUILTIN_OPS:
            a = self.cls_of(node.target)
            if a in ("Mat", "Vec"):
                self.rec(a, "__i" + BUILTIN_OPS[type(node.op)][2:], "operator", node, [node.value])
        self.generic_visit(node)

    def visit_Attribute(self, node):
        # plain attribute reads of petsc4py objects (comm.rank)
        if in_scope(node.lineno, self.ranges) and isinstance(node.ctx, ast.Load):
            rc = self.cls_of(node.value)
            if rc == "Comm" and node.attr in ("rank", "size"):
                self.rec("Comm", node.attr, "attribute", node)
        self.generic_visit(node)

    def visit_ImportFrom(self, node):
        if in_scope(node.lineno, self.ranges) and node.module and node.module.startswith("petsc4py"):
            for a in node.names:
                self.rec("module", a.name, "import", node)
        self.generic_visit(node)


def scan(ref):
    table, unclassified, files = {}, [], []
    for rel, ranges in SCOPE:
        path = os.path.join(ref, rel)
        src = open(path).read()
        tree = ast.parse(src)
        names = set()
        for n in ast.walk(tree):
            if isinstance(n, ast.ImportFrom) and n.module == "petsc4py.PETSc":
                names |= {a.asname or a.name for a in n.names}
        names -= {"COMM_WORLD"}
        s = Scan(rel.split("/")[-1], ranges, names, table)
        for n in ast.walk(tree):  # (the subclasses' own methods, wherever they are called from)
            if isinstance(n, ast.ClassDef) and any(isinstance(b, ast.Name) and b.id in names for b in n.bases):
                s.sub_methods |= {f.name for f in n.body if isinstance(f, ast.FunctionDef)}
        s.visit(tree)
        unclassified += s.unclassified
        files.append({"file": rel, "lines": ranges or "all"})
    for e in table.values():
        e["sites"] = sorted(set(e["sites"]), key=lambda x: (x.split(":")[0], int(x.split(":")[1])))
    return {"generated_by": "tools/scan_petsc4py_surface.py", "scope": files,
            "entries": [table[k] for k in sorted(table)], "unclassified": unclassified}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "tests", "golden", "petsc4py_surface.json"))
    a = ap.parse_args()
    out = scan(a.ref)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out['entries'])} entries, {len(out['unclassified'])} unclassified -> {a.out}")
    for u in out["unclassified"]:
        print("  unclassified:", u)
    return 0


if __name__ == "__main__":
    sys.exit(main())
