"""Writes tests/golden/reference_kats.json.

The numbers are the expected outputs of the reference's own known-answer tests
(medical-genomics-group/rs-bann @ v1), transcribed by hand from the test
modules cited next to each entry.  They are data (inputs + expected outputs),
not code.  The reference values are single-backend ArrayFire f32 results; the
tests compare against them with the per-tensor tolerances documented in
tests/test_oracle_kats.py (SURVEY §0 caveat 2).
"""
import json
import os

KAT = {
    "_source": "medical-genomics-group/rs-bann v1 in-crate unit tests",
    "inputs": {
        "_cite": "src/net/branch/ridge_ard.rs:355-408,457-460,529",
        "x_col_major_4x3": [1., 0., 0., 2., 1., 1., 2., 0., 0., 2., 0., 1.],
        "y": [0.0, 2.0, 1.0, 1.5],
        "w0_col_major_3x2": [0., 1., 2., 3., 4., 5.],
        "w1": [1., 2.], "w_out": [2.], "b0": [0., 1.], "b1": [2.],
        "hyper": {"dense": [3.0, 2.0], "summary": [3.0, 2.0], "output": [4.0, 5.0]},
    },
    # identical in all four prior modules (ridge_ard.rs:474-496, ridge_base.rs:393-415,
    # lasso_ard.rs:473-495, lasso_base.rs:393-415)
    "forward_feed": {
        "a0_col_major": [0.7615942, 0.9999092, 0.9640276, 0.9640276, 0.99999976,
                          0.9999999999998128, 0.99999994, 0.9999999999244973],
        "a1": [0.99985373, 0.99990916, 0.9999024, 0.9999024],
        "out": [1.9997075, 1.9998183, 1.9998049, 1.9998049],
    },
    "rss": 5.248245,
    "ridge_ard": {
        "_cite": "src/net/branch/ridge_ard.rs:520-709",
        "log_density_joint": {"precision": 2.0, "wrt_e": -2.182509, "wrt_w": -57.269924,
                              "wrt_b": -3.1876905, "total": -62.640125},
        "ldg_joint": {
            "precision": 2.0,
            "wrt_w": [[-0.0010378566, -2.00109287e+00, -4.00002756e+00, -6.0, -8.0, -10.0],
                      [-2.0029104, -4.0035105], [-10.997393]],
            "wrt_b": [[-0.0010654309, -2.0], [-4.0035105]],
            "wrt_error_precision": -0.32412243,
            "wrt_w_prec": [[-3.25, -7.25, -13.25], [0.5, -1.0], [-0.45000005]],
            "wrt_b_prec": [0.5, -1.25],
        },
        "ldg": {
            "precision": 1.0,
            "wrt_w": [[-0.0005189283, -1.0005465, -2.0000138, -3.0000000010532997,
                       -4.00000000114826, -5.000000000000059],
                      [-1.0014552, -2.0017552], [-5.4986963]],
            "wrt_b": [[-0.00053271546, -1.2088213e-9], [-0.0017552058]],
        },
    },
    "ridge_base": {
        "_cite": "src/net/branch/ridge_base.rs:420-589",
        "log_density_joint": {"precision": 2.0, "wrt_e": -2.182509, "wrt_w": -58.428806,
                              "wrt_b": -3.1876905, "total": -63.799007},
        "ldg_joint": {
            "precision": 2.0,
            "wrt_w": [[-0.0010378566, -2.00109287e+00, -4.00002756e+00, -6.0, -8.0, -10.0],
                      [-2.0029104, -4.0035105], [-10.997393]],
            "wrt_b": [[-0.0010654309, -2.0], [-4.0035105]],
            "wrt_error_precision": -0.32412243,
            "wrt_w_prec": [[-25.5], [-1.5], [-0.45000005]],
            "wrt_b_prec": [0.5, -1.25],
        },
        "ldg": {
            "precision": 1.0,
            "wrt_w": [[-0.0005189283, -1.0005465, -2.0000138, -3.0, -4.0, -5.0],
                      [-1.0014552, -2.0017552], [-5.4986963]],
            "wrt_b": [[-0.00053271546, -1.2088213e-9], [-0.0017552058]],
        },
    },
    "lasso_ard": {
        "_cite": "src/net/branch/lasso_ard.rs:502-671",
        "log_density_joint": {"precision": 2.0, "wrt_e": -2.182509, "wrt_w": -30.150764,
                              "wrt_b": -3.1876905, "total": -35.520966},
        "ldg_joint": {
            "precision": 2.0,
            "wrt_w": [[-0.0010378566, -2.001093, -2.0000277, -2.0, -2.0, -2.0],
                      [-2.0029104, -2.0035105], [-8.997393]],
            "wrt_b": [[-0.0010654309, -2.0], [-4.0035105]],
            "wrt_error_precision": -0.32412243,
            "wrt_w_prec": [[-1.0, -3.0, -5.0], [0.5, -0.5], [-0.20000005]],
            "wrt_b_prec": [0.5, -1.25],
        },
        "ldg": {
            "precision": 1.0,
            "wrt_w": [[-0.0005189283, -1.0005465, -1.0000138, -1.0000000010532997,
                       -1.00000000114826, -1.000000000000059],
                      [-1.0014552, -1.0017552], [-4.4986963]],
            "wrt_b": [[-0.00053271546, -1.2088213e-9], [-0.0017552058]],
        },
    },
    "lasso_base": {
        "_cite": "src/net/branch/lasso_base.rs:421-606",
        "log_density_joint": {"precision": 2.0, "wrt_e": -2.182509, "wrt_w": -31.309645111040876,
                              "wrt_b": -3.1876905, "total": -36.67984440609501},
        "ldg_joint": {
            "precision": 2.0,
            "wrt_w": [[-0.0010378566, -2.001093, -2.0000277, -2.0, -2.0, -2.0],
                      [-2.0029104, -2.0035105], [-8.997393]],
            "wrt_b": [[-0.0010654309, -2.0], [-4.0035105]],
            "wrt_error_precision": -0.32412243,
            "wrt_w_prec": [[-11.5], [-1.5], [-0.20000005]],
            "wrt_b_prec": [0.5, -1.25],
        },
        "log_density": {"precision": 2.0, "wrt_e": -5.24824469, "wrt_w": -40.0,
                        "_note": "lasso_base.rs:538-571; wrt_b_l2 is log_density_wrt_biases_l2, not part of total",
                        "wrt_b_l2": -5.0, "total": -45.24824469},
        "ldg": {
            "precision": 2.0,
            "wrt_w": [[-0.0010378566, -2.001093, -2.0000277, -2.0, -2.0, -2.0],
                      [-2.0029104, -2.0035105], [-8.997393]],
            "wrt_b": [[-0.0010654309, -2.4176425e-9], [-0.0035104116]],
        },
    },
    "params_param_vec": {
        "_cite": "src/net/params.rs:777-795",
        "weights": [[0.1, 0.2], [0.3]], "biases": [[0.4]], "num_markers": 2, "layer_widths": [1, 1],
        "expected": [0.1, 0.2, 0.3, 0.4],
    },
    "bed_small": {
        "_cite": "src/io/bed.rs:430-497; resources/test/README.md:7-31",
        "n": 20, "m": 11,
        "bed_payload_hex": None,  # filled from resources/test/small.bed by the generator below
        "data_f32_col_major": [
            0., 0., 1., 0., 1., 0., 0., 1., 0., 0., 1., 0., 0., 0., 0., 0., 1., 0., 2., 0., 1., 0.,
            1., 0., 0., 2., 0., 0., 1., 1., 1., 1., 0., 0., 0., 1., 0., 0., 1., 0., 0., 0., 0., 0.,
            0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 1., 0., 0., 0., 0., 0., 0., 1., 0., 0., 0., 1.,
            1., 0., 0., 0., 1., 0., 0., 0., 1., 0., 0., 0., 1., 1., 0., 0., 0., 0., 0., 0., 0., 0.,
            0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 2., 0., 1., 1., 1., 2., 0., 1., 1.,
            1., 1., 2., 0., 0., 1., 2., 1., 0., 1., 2., 0., 1., 0., 0., 0., 1., 0., 0., 0., 0., 1.,
            1., 0., 0., 0., 0., 1., 1., 1., 1., 1., 0., 1., 1., 1., 1., 0., 1., 0., 1., 2., 2., 1.,
            1., 1., 2., 1., 1., 1., 0., 0., 0., 0., 0., 2., 0., 0., 0., 0., 0., 1., 0., 0., 0., 2.,
            0., 0., 0., 0., 0., 1., 0., 1., 1., 2., 0., 0., 0., 0., 1., 1., 1., 1., 1., 1., 1., 1.,
            1., 0., 1., 1., 0., 1., 1., 0., 1., 0., 0., 2., 1., 1., 1., 1., 0., 0., 1., 1., 0., 0.],
        "col_means": [0.35, 0.5, 0.05, 0.35, 0., 0.9, 0.45, 1., 0.25, 0.7, 0.65],
        "col_stds": [0.5722761, 0.591608, 0.21794495, 0.47696957, 0.0, 0.70000005, 0.58949125,
                     0.5477226, 0.622495, 0.55677646, 0.5722762],
        "submatrix_cols": [0, 5],
        "submatrix_standardized": [
            -0.6115929, -0.6115929, 1.1358153, -0.6115929, 1.1358153, -0.6115929, -0.6115929,
            1.1358153, -0.6115929, -0.6115929, 1.1358153, -0.6115929, -0.6115929, -0.6115929,
            -0.6115929, -0.6115929, 1.1358153, -0.6115929, 2.8832235, -0.6115929, -1.2857141,
            1.5714285, -1.2857141, 0.14285716, 0.14285716, 0.14285716, 1.5714285, -1.2857141,
            0.14285716, 0.14285716, 0.14285716, 0.14285716, 1.5714285, -1.2857141, -1.2857141,
            0.14285716, 1.5714285, 0.14285716, -1.2857141, 0.14285716],
        "chunkf32_to_byte": {"_cite": "src/io/bed.rs:414-416", "input": [1., 0., 1., 1.], "expected": 174},
    },
    "architecture_num_params": {
        "_cite": "branch_builder.rs build_branch_success (12), branch_cfg_builder.rs:406-418 (17), architectures.rs:245-256 (22)",
        "branch_builder_m3_w2": 12,
    },
}

if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    bed = "/root/reference/resources/test/small.bed"
    with open(bed, "rb") as f:
        raw = f.read()
    assert raw[:3] == bytes([0x6C, 0x1B, 0x01]), "variant-major .bed signature"
    KAT["bed_small"]["bed_payload_hex"] = raw[3:].hex()
    with open(os.path.join(here, "reference_kats.json"), "w") as f:
        json.dump(KAT, f, indent=1)
    print("wrote reference_kats.json")
