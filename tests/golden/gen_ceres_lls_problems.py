"""Writes tests/golden/ceres_lls_problems.json: the block-sparse linear least-squares fixtures the
reference's vendored Ceres 2.0 holds for its Schur tests, restated as data (the C++ file cannot be
compiled here: it needs Eigen).  Source: /root/reference/thirdparty/ceres-solver/internal/ceres/
linear_least_squares_problems.cc — LinearLeastSquaresProblem2 (:288-419, scalar blocks, 2 e-blocks),
LinearLeastSquaresProblem3 (:421-518, every column eliminated) and LinearLeastSquaresProblem4
(:520-600, f-blocks of sizes 3 and 2, one e-block of size 2).  b[i] = i; D as each problem sets it.
Used by tests/test_oracle.py with the checks of schur_eliminator_test.cc:196-225 and
schur_complement_solver_test.cc:50-220.

    python tests/golden/gen_ceres_lls_problems.py
"""
import json
import os

# each row block: [row_size, [[col_block, [row-major values]], ...]]
P2 = {"col_sizes": [1, 1, 1, 1, 1], "num_eliminate_blocks": 2,
      "rows": [[1, [[0, [1]], [2, [2]]]],
               [1, [[0, [3]], [3, [4]]]],
               [1, [[1, [5]], [4, [6]]]],
               [1, [[1, [7]], [2, [8]]]],
               [1, [[1, [9]], [2, [1]]]],
               [1, [[2, [1]], [3, [1]], [4, [1]]]]],
      "D": [1, 1, 1, 1, 1]}
P3 = {"col_sizes": [1, 1], "num_eliminate_blocks": 2,
      "rows": [[1, [[0, [1]]]], [1, [[0, [3]]]], [1, [[1, [5]]]], [1, [[1, [7]]]], [1, [[1, [9]]]]],
      "D": [1, 1]}
P4 = {"col_sizes": [2, 3, 2], "num_eliminate_blocks": 1,
      "rows": [[2, [[0, [1, 2, 1, 4]], [2, [1, 1, 5, 6]]]],
               [1, [[1, [9, 0, 0]], [2, [3, 1]]]]],
      "D": [(i + 1) * 100 for i in range(7)]}

if __name__ == "__main__":
    out = {}
    for name, pr in (("problem2", P2), ("problem3", P3), ("problem4", P4)):
        nrows = sum(r[0] for r in pr["rows"])
        out[name] = dict(pr, b=list(range(nrows)))
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "ceres_lls_problems.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", list(out))
