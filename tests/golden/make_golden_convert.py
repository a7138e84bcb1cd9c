"""Golden fixture for the caffemodel -> npz converter's copy lists, extracted from the
REFERENCE's own converter source without running it.

Run in the build container only (needs /root/reference, absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_convert.py

models/convert_model.py:8-249 keeps, per architecture, the list of layer names whose W / b it copies
out of the caffemodel.  The module cannot be imported here (it imports chainer and chainer.links.caffe
at the top), so the `layer_names` dict literal is read with `ast.literal_eval` from the parsed source:
nothing of the reference executes.  Writes tests/golden/convert_layer_names.json (data only: arch ->
ordered list of names).
"""
import ast
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/models/convert_model.py"


def extract(path=SRC):
    tree = ast.parse(open(path).read(), filename=path)
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "layer_names" for t in node.targets):
            return ast.literal_eval(node.value), node.lineno, node.end_lineno
    raise SystemExit("layer_names not found in " + path)


if __name__ == "__main__":
    table, l0, l1 = extract()
    out = {"source": "models/convert_model.py:%d-%d" % (l0, l1), "layer_names": table}
    with open(os.path.join(HERE, "convert_layer_names.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: len(v) for k, v in table.items()}, out["source"])
