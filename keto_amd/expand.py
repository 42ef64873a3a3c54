"""expand.Engine — BuildTree over the snapshot, and the expand.Tree model.

Mirrors internal/expand/engine.go:30-98 (BuildTree) and internal/expand/tree.go
(NodeType, Tree, JSON codec :85-91,156-162).  BuildTree's output order depends on
the backend's row order, so it is a sequential walk of the snapshot's ordered rows
(host_engine.cpp), not a GPU traversal.
"""
import ctypes as C
import json
from dataclasses import dataclass, field
from typing import List, Optional

from . import _lib as L
from .relationtuple import Subject, SubjectID, SubjectSet
from .snapshot import Snapshot, subject_struct

Union, Exclusion, Intersection, Leaf = "union", "exclusion", "intersection", "leaf"



def _depth(d):
    """restDepth for the int32 argument of ketogpu_expand: every depth <= 0 is the nil
    tree and every depth beyond INT32_MAX exceeds any tree's height, so clamping keeps
    BuildTree's answer (ctypes would silently truncate a wider Go int)"""
    return max(-1, min(int(d), 2**31 - 1))

class NotFound(LookupError):
    """herodot.ErrNotFound (HTTP 404)"""


@dataclass
class Tree:
    type: str
    subject: Subject
    children: List["Tree"] = field(default_factory=list)

    def to_node(self):
        """the JSON `node` of tree.go:85-91 (children omitempty)"""
        d = {"type": self.type}
        if self.children:
            d["children"] = [c.to_node() for c in self.children]
        d.update(self.subject.to_dict())
        return d

    def MarshalJSON(self) -> str:
        return json.dumps(self.to_node(), separators=(",", ":"))


def _subject(s: L.Subject) -> Subject:
    if s.kind == L.SUBJECT_ID:
        return SubjectID(s.id.decode("utf-8"))
    return SubjectSet(s.ns.decode("utf-8"), s.obj.decode("utf-8"), s.rel.decode("utf-8"))


class Engine:
    def __init__(self, snapshot: Snapshot):
        self.L = L.lib()
        self.snapshot = snapshot

    def tree_size(self, subject: Subject, rest_depth: int) -> int:
        """number of nodes of BuildTree's tree (0 for a nil tree), built and dropped in C++
        without Python objects (throughput measurements)"""
        h = C.c_void_p()
        subj = subject_struct(subject)
        rc = self.L.ketogpu_expand(self.snapshot.h, C.byref(subj), _depth(rest_depth), C.byref(h))
        if rc == L.ENOTFOUND:
            raise NotFound(self.L.ketogpu_last_error().decode("utf-8", "replace"))
        L.check(rc)
        if not h.value:
            return 0
        try:
            nodes = C.POINTER(L.TreeNode)()
            n = C.c_size_t()
            L.check(self.L.ketogpu_tree_nodes(h, C.byref(nodes), C.byref(n)))
            return int(n.value)
        finally:
            self.L.ketogpu_tree_free(h)

    def BuildTree(self, subject: Subject, rest_depth: int) -> Optional[Tree]:
        h = C.c_void_p()
        subj = subject_struct(subject)
        rc = self.L.ketogpu_expand(self.snapshot.h, C.byref(subj), _depth(rest_depth), C.byref(h))
        if rc == L.ENOTFOUND:
            raise NotFound(self.L.ketogpu_last_error().decode("utf-8", "replace"))
        L.check(rc)
        if not h.value:
            return None
        try:
            nodes = C.POINTER(L.TreeNode)()
            n = C.c_size_t()
            L.check(self.L.ketogpu_tree_nodes(h, C.byref(nodes), C.byref(n)))
            pos = 0

            def take():
                nonlocal pos
                nd = nodes[pos]
                pos += 1
                t = Tree(Leaf if nd.type == L.NODE_LEAF else Union, _subject(nd.subject))
                for _ in range(nd.num_children):
                    t.children.append(take())
                return t

            return take()
        finally:
            self.L.ketogpu_tree_free(h)

    build_tree = BuildTree

    def build_tree_json(self, subject: Subject, rest_depth: int) -> str:
        """the library's own MarshalJSON (ketogpu_tree_json)"""
        h = C.c_void_p()
        subj = subject_struct(subject)
        rc = self.L.ketogpu_expand(self.snapshot.h, C.byref(subj), _depth(rest_depth), C.byref(h))
        if rc == L.ENOTFOUND:
            raise NotFound(self.L.ketogpu_last_error().decode("utf-8", "replace"))
        L.check(rc)
        out = C.c_void_p()
        try:
            L.check(self.L.ketogpu_tree_json(h if h.value else None, C.byref(out)))
            s = C.string_at(out.value).decode("utf-8")
            self.L.ketogpu_free(out)
            return s
        finally:
            if h.value:
                self.L.ketogpu_tree_free(h)
