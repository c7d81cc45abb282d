"""sng-render (synerfgine_amd/csrc/sng_render.cpp), the headless CLI of SURVEY.md §8(b): the reference's
render flags (main.cu:44-133) parsed the way its args::ArgumentParser does, so the command line of
scripts/render/profiling.sh:18 runs against this library with only EXEC swapped.  CPU: --dry-run parses and
prints the options without touching the GPU."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "synerfgine_amd", "_build", "sng-render")


@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(CLI):
        r = subprocess.run(["make", "-C", os.path.join(REPO, "synerfgine_amd"), "-j8"], capture_output=True, text=True)
        if r.returncode != 0 or not os.path.exists(CLI):
            pytest.skip("sng-render not buildable here: " + r.stderr[-400:])
    return CLI


def run(cli, *args):
    return subprocess.run([cli, *args], capture_output=True, text=True, timeout=60)


def test_profiling_sh_command_line(cli):
    # scripts/render/profiling.sh:18 with ROOT="..", FOLDER=dmrf-compare-abm, NERF=lego, SSHADOW=2, NSHADOW=4
    r = run(cli, "--dry-run", "--snapshot", "../data/nerf/lego.ingp", "--virtual", "../scripts/virtual_desc/dmrf-compare-abm.json",
            "--frag", "../scripts/virtual_desc/main.frag", "--width", "1280", "--height", "720", "--sshadows", "2", "--nshadows", "4")
    assert r.returncode == 0, r.stderr
    o = json.loads(r.stdout)
    assert o["snapshot"] == "../data/nerf/lego.ingp" and o["virtual"] == "../scripts/virtual_desc/dmrf-compare-abm.json"
    assert (o["width"], o["height"], o["sshadows"], o["nshadows"]) == (1280, 720, 2, 4)
    assert o["frag"].endswith("main.frag") and o["frames"] == 1 and o["gpus"] == 1


def test_aliases_equals_form_and_headless_flags(cli):
    r = run(cli, "--dry-run", "--load_snapshot=a.ingp", "--rt", "s.json", "--width=640", "--height=360", "--frames", "3", "--out", "o",
            "--gpus", "8", "--balance", "2", "--set", "rt_tile=4", "--set=nerf_spec_rounds=2", "--display")
    o = json.loads(r.stdout)
    assert (o["snapshot"], o["virtual"], o["width"], o["height"]) == ("a.ingp", "s.json", 640, 360)
    assert (o["frames"], o["out"], o["gpus"], o["balance"], o["display"]) == (3, "o", 8, 2, True)
    assert o["sets"] == {"rt_tile": 4.0, "nerf_spec_rounds": 2.0}
    assert o["sshadows"] == -1   # not given: the engine keeps the scene JSON's values (main.cu:210)


def test_positional_files_like_load_file(cli):
    o = json.loads(run(cli, "--dry-run", "x/lego.ingp", "scene.json").stdout)
    assert o["snapshot"] == "x/lego.ingp" and o["virtual"] == "scene.json"


@pytest.mark.parametrize("args", [["--bogus"], ["--width"], ["--width", "wide"], ["--gpus", "0"], ["--set", "novalue"], ["model.obj"]])
def test_parse_errors_exit_nonzero_with_usage(cli, args):
    r = run(cli, *args)
    assert r.returncode == 2 and "--snapshot" in r.stderr


def test_help_and_version(cli):
    assert run(cli, "--help").returncode == 0 and "--sshadows" in run(cli, "-h").stdout
    r = run(cli, "--version")
    assert r.returncode == 0 and "ABI" in r.stdout
