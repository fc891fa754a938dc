import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bidirectional-pathtracing_amd"), os.path.join(REPO, "tests")]
import bdpt_amd as B
G = os.path.join(REPO, "tests/golden/scenes")
E = json.load(open(f"{G}/CBempty.json")); S = json.load(open(f"{G}/CBspheres.json"))
variants = {"empty": E, "spheres": S,
            "empty+area": dict(E, lights=S["lights"]), "spheres+point": dict(S, lights=E["lights"])}
emp_nomat = dict(E); emp_nomat["materials"] = [m if m["type"] != "emission" else {"type": "diffuse", "reflectance": [0.6, 0.6, 0.6]} for m in E["materials"]]
variants["empty-noemis"] = emp_nomat
for name, js in variants.items():
    sc = B.retarget_camera(B.scene_from_json(js), 480, 360)
    pt = B.BidirectionalPathTracer(sc, 480, 360, 32, 5, seed=5489)
    pt.raytrace_tiles([], 0, 1); pt.sync(); pt.clear()
    t0 = time.perf_counter(); pt.raytrace_tiles([], 0, 32); pt.sync(); dt = time.perf_counter() - t0
    print(f"{name:16s} {480*360*32/dt/1e6:8.1f} Msamples/s", flush=True)
    pt.close()
