"""The library's own scene-file reader (rt_load_yaml_scene, initialize() of main.cu:623-786)
against the Python host layer's PyYAML loader (scene.py). Both must build byte-identical
scene tables (rt_scene_digest). The reference reads the files with yaml-cpp 0.7.0, whose
binary is not in the reference tree. PyYAML 6 is the parser the fixtures were checked
with. Runs on CPU: device -1 contexts build and commit scenes without a GPU."""
import glob
import os

import pytest
import yaml

import raytracingthenextweekcuda_amd as rtmi
from raytracingthenextweekcuda_amd.scene import MODELS_DIR, SCENES_DIR

SCENE_FILES = sorted(f for f in glob.glob(os.path.join(SCENES_DIR, "*.yaml")) if not f.endswith("scene.yaml"))


def _python_digest(path, w, h):
    r = rtmi.Renderer(-1)
    try:
        rtmi.load_yaml_scene(r, path, w, h)
        return r.scene_digest(), r.object_counts()
    finally:
        r.close()


def _native_digest(path, w, h):
    r = rtmi.Renderer(-1)
    try:
        r.load_yaml_native(path, w, h, MODELS_DIR)
        r.commit()
        return r.scene_digest(), r.object_counts()
    finally:
        r.close()


@pytest.mark.parametrize("path", SCENE_FILES, ids=os.path.basename)
@pytest.mark.parametrize("w,h", [(512, 512), (1280, 720)])
def test_native_reader_builds_the_same_scene(path, w, h):
    assert _native_digest(path, w, h) == _python_digest(path, w, h)


@pytest.mark.parametrize("true_word,false_word", [("yes", "no"), ("On", "Off"), ("TRUE", "False")])
def test_native_reader_yaml11_booleans(tmp_path, true_word, false_word):
    # twoSide spelled with other YAML 1.1 booleans: PyYAML and the reader agree
    src = os.path.join(SCENES_DIR, "cornellbox1.yaml")
    text = open(src).read().replace("twoSide: true", f"twoSide: {true_word}")
    text = text.replace("twoSide: false", f"twoSide: {false_word}")
    p = tmp_path / "b.yaml"
    p.write_text(text)
    assert yaml.safe_load(text) == yaml.safe_load(open(src).read())
    assert _native_digest(str(p), 64, 64) == _python_digest(src, 64, 64)


def test_digest_sees_the_camera_aspect():
    path = os.path.join(SCENES_DIR, "cornellbox1.yaml")
    assert _native_digest(path, 512, 512)[0] != _native_digest(path, 640, 512)[0]


@pytest.mark.parametrize("style", ["flow_leaves", "indent4", "doc_marker_and_comments", "same_indent_lists"])
def test_native_reader_layout_variants(tmp_path, style):
    """The same document in other YAML layouts (flow leaf lists, deeper indentation, a
    `---` header and comments, lists at their key's column) gives the same scene."""
    src = os.path.join(SCENES_DIR, "cornellbox2.yaml")
    with open(src) as fh:
        doc = yaml.safe_load(fh)
    if style == "flow_leaves":
        text = yaml.safe_dump(doc, default_flow_style=None, sort_keys=False)
        assert "[" in text
    elif style == "indent4":
        text = yaml.safe_dump(doc, default_flow_style=False, sort_keys=False, indent=4)
    elif style == "doc_marker_and_comments":
        body = yaml.safe_dump(doc, default_flow_style=False, sort_keys=False)
        text = "---\n# leading comment\n" + "\n".join(ln + "   # trailing" if ln.endswith(":") else ln
                                                     for ln in body.splitlines()) + "\n"
    else:
        text = yaml.safe_dump(doc, default_flow_style=False, sort_keys=False, indent=2)
        assert any(ln.lstrip().startswith("- ") for ln in text.splitlines())
    assert yaml.safe_load(text) == doc
    p = tmp_path / f"{style}.yaml"
    p.write_text(text)
    assert _native_digest(str(p), 300, 200) == _python_digest(src, 300, 200)


def _native_error(path):
    r = rtmi.Renderer(-1)
    try:
        with pytest.raises(rtmi.RTError) as e:
            r.load_yaml_native(path, 64, 64, MODELS_DIR)
        return str(e.value)
    finally:
        r.close()


def test_reference_scene_yaml_is_rejected_with_its_line():
    # resources/scenes/scene.yaml ends with a plane that has no extend/material:
    # yaml-cpp throws on it in the reference; the Python loader raises KeyError
    path = os.path.join(SCENES_DIR, "scene.yaml")
    with pytest.raises(KeyError):
        _python_digest(path, 64, 64)
    msg = _native_error(path)
    assert "RT_ERR_INVALID" in msg and "line 167:" in msg


@pytest.mark.parametrize("text,needle", [
    ("camera:\n\teye: [0, 0, 1]\n", "tab indentation"),
    ("camera:\n  eye [0, 0, 1]\n", "expected 'key: value'"),
    ("camera: &a\n  eye: [0, 0, 1]\n", "unsupported"),
    ("camera:\n  fov: 60\n  fov: 30\n", "duplicate key"),
    ("camera:\n  eye: [0, 0, 1]\n  center: [0, 0, -1]\n  up: [0, 1, 0]\n  fov: 60\n  aperture: 0\n"
     "objects:\n  - thing:\n      type: 9\n      materialId: 3\n      material:\n        type: 0\n"
     "        albedo: [1, 1, 1]\n", "unknown primitive type 9"),
    ("camera:\n  eye: [0, 0]\n", "camera needs"),
])
def test_native_reader_errors_name_the_problem(tmp_path, text, needle):
    p = tmp_path / "bad.yaml"
    p.write_text(text)
    msg = _native_error(str(p))
    assert needle in msg and "line" in msg, msg


def test_missing_scene_file_is_an_io_error():
    assert "RT_ERR_IO" in _native_error("/nonexistent/scene.yaml")


def test_reader_survives_mutation_fuzzing_under_sanitizers(tmp_path):
    """Host-code sanitizers (ASan + UBSan) over the reader with random mutations of
    every scene file and hostile nesting (tools/yaml_fuzz.cpp)."""
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "yaml_fuzz"
    subprocess.run(["g++", "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I" + os.path.join(repo, "raytracingthenextweekcuda_amd", "csrc"),
                    os.path.join(repo, "tools", "yaml_fuzz.cpp"),
                    os.path.join(repo, "raytracingthenextweekcuda_amd", "csrc", "rt_yaml.cpp"), "-o", str(exe)],
                   check=True)
    files = sorted(glob.glob(os.path.join(SCENES_DIR, "*.yaml")))
    out = subprocess.run([str(exe), "400"] + files, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "mutants parsed" in out.stdout
