"""Summarise rocprofv3 PMC passes (tools/pmc.sh output) into
profiles/pmc_traffic.json: per kernel, HBM-side bytes per launch.

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE / WRITE_SIZE are in KB and
derive from the L2's memory-side request counters; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled here;
WRITE_SIZE is taken as is.  Usage: python tools/pmc_summary.py PMC_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import sys

SHORT = {"k_normals_stile": "normals_stile", "k_normals_vlist": "normals_stile", "k_normals_knn_tile": "normals_tile", "k_normals_knn_wave": "normals_wave",
         "k_voxel_assign_dense": "voxel_assign", "k_icp_accumulate": "icp_accumulate",
         "k_icp_match": "icp_match", "k_icp_step": "icp_step", "k_icp_moments": "icp_moments", "k_vbin_scatter": "vbin_scatter",
         "k_plane_count": "plane_count", "k_plane_fixup": "plane_fixup", "k_grid_count": "grid_count", "k_grid_cell_sort": "grid_sort",
         "k_vbin_count": "vbin_count", "k_vbin_reduce": "vbin_reduce", "k_gather_vox": "gather_vox",
         "k_aabb_partial": "aabb_partial", "k_tile_compact_u8": "compact_u8",
         "k_vbin_fused": "vbin_fused", "k_plane_upper": "plane_upper", "k_icp_match": "icp_match"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def main(src, out):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            if k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"source": "rocprofv3 --pmc, one counter group per pass (tools/pmc.sh); "
                     "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KB -> B, gfx950 FETCH correction)",
           "kernels": {}}
    for k, d in sorted(vals.items()):
        e = {c: sum(v) / len(v) for c, v in d.items()}
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = 2.0 * e["FETCH_SIZE"] * 1024 + e["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in e and "SQ_WAVES" in e:
            # VALU-issue floor: a wave64 VALU instruction issues in 2 cycles on a
            # SIMD holding >= 2 waves (MI355X_MICROARCH.md), 1024 SIMDs (256 CUs
            # x 4) at the 2.4 GHz peak engine clock; float64 / packed /
            # transcendental instructions take longer, so this is a lower bound
            e["valu_insts_per_wave"] = e["SQ_INSTS_VALU"] / e["SQ_WAVES"]
            e["valu_issue_floor_ms"] = e["SQ_INSTS_VALU"] * 2.0 / (1024 * 2.4e9) * 1e3
        if "SQ_ACTIVE_INST_VALU" in e and "SQ_WAVE_CYCLES" in e:
            e["valu_active_frac_of_wave_cycles"] = e["SQ_ACTIVE_INST_VALU"] / e["SQ_WAVE_CYCLES"]
        e["launches_sampled"] = max(len(v) for v in d.values())
        res["kernels"][k] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in res["kernels"].items()}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
