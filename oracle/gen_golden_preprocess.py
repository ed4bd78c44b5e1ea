"""TEST INFRASTRUCTURE - writes tests/golden/preprocess_kat.npz from the reference's own loader code.

The reference's dataset modules cannot be imported here (torchvision / imageio are absent), so
this script reads their source text, takes out the pieces of the label / image transform - the
id_to_trainid tables and 16/13-class sets of each loader's __init__, and the bodies of
City_Dataset.id2trainId / _img_transform (datasets/cityscapes_Dataset.py:124-155, 245-251; the
GTA5 and SYNTHIA loaders subclass it with their own tables, gta5_Dataset.py:73-75,
synthia_Dataset.py:56-62) - and runs those functions, unmodified, on synthetic uint8 images and
id maps.  Only the resulting vectors are committed; no reference source enters the repository.
Runs in the survey container only (skips when /root/reference is absent).
"""
import argparse
import ast
import os
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _class(tree, name):
    return next(n for n in ast.walk(tree) if isinstance(n, ast.ClassDef) and n.name == name)


def _method(cls, name):
    return next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == name)


def _self_assign(fn, attr, src, env):
    """Evaluate the value expression of `self.<attr> = ...` inside method `fn`."""
    for node in ast.walk(fn):
        if isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Attribute) and t.attr == attr for t in node.targets):
            return eval(compile(ast.Expression(node.value), "<ref>", "eval"), dict(env))
    raise KeyError(attr)


def _local_assign(fn, name, env):
    for node in ast.walk(fn):
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == name for t in node.targets):
            return eval(compile(ast.Expression(node.value), "<ref>", "eval"), dict(env))
    raise KeyError(name)


def _function(fn_node, env):
    mod = ast.Module(body=[fn_node], type_ignores=[])
    ns = dict(env)
    exec(compile(mod, "<ref>", "exec"), ns)
    return ns[fn_node.name]


def load(ref_root):
    ds = os.path.join(ref_root, "datasets")
    trees = {k: ast.parse(open(os.path.join(ds, f)).read()) for k, f in
             (("city", "cityscapes_Dataset.py"), ("gta5", "gta5_Dataset.py"), ("synthia", "synthia_Dataset.py"))}
    env = {"np": np, "torch": torch}
    # module-level IMG_MEAN of cityscapes_Dataset.py:14
    for node in trees["city"].body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "IMG_MEAN" for t in node.targets):
            env["IMG_MEAN"] = eval(compile(ast.Expression(node.value), "<ref>", "eval"), dict(env))
    city = _class(trees["city"], "City_Dataset")
    id2train = _function(_method(city, "id2trainId"), env)
    img_tf = _function(_method(city, "_img_transform"), env)
    tables = {}
    for key, cname in (("cityscapes", "City_Dataset"), ("gta5", "GTA5_Dataset"), ("synthia", "SYNTHIA_Dataset")):
        init = _method(_class(trees["city" if key == "cityscapes" else key], cname), "__init__")
        e = dict(env, ignore_label=-1)
        tables[key] = _self_assign(init, "id_to_trainid", None, e)
    init = _method(city, "__init__")
    set16 = _local_assign(init, "synthia_set_16", env)
    set13 = _local_assign(init, "synthia_set_13", env)
    return env["IMG_MEAN"], id2train, img_tf, tables, set16, set13


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(HERE), "tests", "golden"))
    a = ap.parse_args()
    if not os.path.isdir(a.ref):
        print("reference not present; goldens are committed, nothing to do")
        return
    mean, id2train, img_tf, tables, set16, set13 = load(a.ref)
    rng = np.random.default_rng(2024)
    out = {"img_mean": np.asarray(mean, np.float32)}
    for tag, (h, w) in (("a", (37, 52)), ("b", (16, 24)), ("c", (9, 13))):
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        # mostly the labelled id range 0..34, the rest anywhere in 0..255
        ids = np.where(rng.random((h, w)) < 0.7, rng.integers(0, 35, (h, w)), rng.integers(0, 256, (h, w))).astype(np.uint8)
        ids.reshape(-1)[: 64] = np.arange(64, dtype=np.uint8)  # every low id appears
        out[f"{tag}_rgb"], out[f"{tag}_ids"] = rgb, ids
        for mirror in (0, 1):
            r = rgb[:, ::-1] if mirror else rgb       # Image.FLIP_LEFT_RIGHT (cityscapes_Dataset.py:182-183)
            d = ids[:, ::-1] if mirror else ids
            fake = types.SimpleNamespace(args=types.SimpleNamespace(numpy_transform=True))
            out[f"{tag}_m{mirror}_img"] = img_tf(fake, r).numpy()
            for ds, t in tables.items():
                for c16, c13 in ((False, False), (True, False), (False, True)):
                    if ds == "synthia" and c13:
                        continue
                    s = types.SimpleNamespace(id_to_trainid=t, class_16=c16, class_13=c13,
                                              trainid_to_16id={i: k for k, i in enumerate(set16)},
                                              trainid_to_13id={i: k for k, i in enumerate(set13)})
                    lab = id2train(s, np.asarray(d, np.float32))
                    out[f"{tag}_m{mirror}_{ds}_{'16' if c16 else '13' if c13 else '19'}"] = lab.astype(np.float32)
    np.savez_compressed(os.path.join(a.out, "preprocess_kat.npz"), **out)
    print("wrote", sorted(out)[:6], "...", len(out), "arrays")


if __name__ == "__main__":
    main()
