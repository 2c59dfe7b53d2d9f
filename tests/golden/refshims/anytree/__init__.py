"""Minimal stand-in for the `anytree` package (only used to IMPORT the reference here).

Provides just the NodeMixin surface the reference MCTS touches (`parent`,
`children`, `is_leaf`, `_post_detach_children`), keeping child order = attach
order like anytree 2.8.  Test infrastructure only; never shipped or imported by
the product package.
"""


class NodeMixin:
    @property
    def parent(self):
        return self.__dict__.get("_nm_parent")

    @parent.setter
    def parent(self, value):
        old = self.__dict__.get("_nm_parent")
        if old is value:
            return
        if old is not None:
            old.__dict__["_nm_children"] = [c for c in old.__dict__.get("_nm_children", []) if c is not self]
        self.__dict__["_nm_parent"] = value
        if value is not None:
            value.__dict__.setdefault("_nm_children", []).append(self)

    @property
    def children(self):
        return tuple(self.__dict__.get("_nm_children", []))

    @children.setter
    def children(self, new_children):
        new_children = list(new_children)
        old = list(self.__dict__.get("_nm_children", []))
        for c in old:
            if not any(c is n for n in new_children):
                c.__dict__["_nm_parent"] = None
        if hasattr(self, "_post_detach_children"):
            self._post_detach_children(tuple(old))
        self.__dict__["_nm_children"] = []
        for c in new_children:
            prev = c.__dict__.get("_nm_parent")
            if prev is not None and prev is not self:
                prev.__dict__["_nm_children"] = [x for x in prev.__dict__.get("_nm_children", []) if x is not c]
            c.__dict__["_nm_parent"] = self
            self.__dict__["_nm_children"].append(c)

    @property
    def is_leaf(self):
        return len(self.__dict__.get("_nm_children", [])) == 0
