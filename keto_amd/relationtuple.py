"""Relation-tuple data model, mirroring internal/relationtuple/definitions.go.

SubjectID / SubjectSet / InternalRelationTuple keep the reference's names, string
codecs and typed equality:
  SubjectFromString            definitions.go:138-143
  SubjectID.String / FromString definitions.go:164-175
  SubjectSet.String / FromString definitions.go:168-193
  Equals                       definitions.go:253-267
  InternalRelationTuple.String / FromString definitions.go:273-306
"""
from dataclasses import dataclass
from typing import Optional, Union


class MalformedInput(ValueError):
    """relationtuple.ErrMalformedInput"""


class NilSubject(ValueError):
    """relationtuple.ErrNilSubject"""


@dataclass(frozen=True)
class SubjectID:
    id: str

    def String(self) -> str:
        return self.id

    def Equals(self, other) -> bool:
        return isinstance(other, SubjectID) and other.id == self.id

    def to_dict(self):
        return {"subject_id": self.id}


@dataclass(frozen=True)
class SubjectSet:
    namespace: str = ""
    object: str = ""
    relation: str = ""

    def String(self) -> str:
        return f"{self.namespace}:{self.object}#{self.relation}"

    def Equals(self, other) -> bool:
        return (isinstance(other, SubjectSet) and other.relation == self.relation and other.object == self.object
                and other.namespace == self.namespace)

    @staticmethod
    def FromString(s: str) -> "SubjectSet":
        parts = s.split("#")
        if len(parts) != 2:
            raise MalformedInput(s)
        inner = parts[0].split(":")
        if len(inner) != 2:
            raise MalformedInput(s)
        return SubjectSet(inner[0], inner[1], parts[1])

    def to_dict(self):
        return {"subject_set": {"namespace": self.namespace, "object": self.object, "relation": self.relation}}


Subject = Union[SubjectID, SubjectSet]


def SubjectFromString(s: str) -> Subject:
    if "#" in s:
        return SubjectSet.FromString(s)
    return SubjectID(s)


def subject_from_dict(d) -> Optional[Subject]:
    if d.get("subject_id") is not None:
        return SubjectID(d["subject_id"])
    if d.get("subject_set") is not None:
        s = d["subject_set"]
        return SubjectSet(s.get("namespace", ""), s.get("object", ""), s.get("relation", ""))
    return None


@dataclass
class InternalRelationTuple:
    namespace: str = ""
    object: str = ""
    relation: str = ""
    subject: Optional[Subject] = None

    def String(self) -> str:
        return f"{self.namespace}:{self.object}#{self.relation}@{self.subject.String() if self.subject else '<nil>'}"

    @staticmethod
    def FromString(s: str) -> "InternalRelationTuple":
        parts = s.split(":", 1)
        if len(parts) != 2:
            raise MalformedInput("expected input to contain ':'")
        ns = parts[0]
        parts = parts[1].split("#", 1)
        if len(parts) != 2:
            raise MalformedInput("expected input to contain '#'")
        obj = parts[0]
        parts = parts[1].split("@", 1)
        if len(parts) != 2:
            raise MalformedInput("expected input to contain '@'")
        rel = parts[0]
        sub = parts[1].strip("()")
        return InternalRelationTuple(ns, obj, rel, SubjectFromString(sub))

    @staticmethod
    def from_dict(d) -> "InternalRelationTuple":
        return InternalRelationTuple(d.get("namespace", ""), d.get("object", ""), d.get("relation", ""),
                                     subject_from_dict(d))

    def to_dict(self):
        d = {"namespace": self.namespace, "object": self.object, "relation": self.relation}
        if self.subject is not None:
            d.update(self.subject.to_dict())
        return d
