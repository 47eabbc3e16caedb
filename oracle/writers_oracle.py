"""The reference's result-file loops restated with csv.writer — TEST INFRASTRUCTURE ONLY
(workflow_viterbi.py:690-743, workflow_posterior.py:697-716; the workflow modules cannot be
imported here: their _version module is generated at install time)."""
import csv


def viterbi_csv(output_file, viterbi_result, ref_coordinates=None):
    with open(output_file, "w", newline="") as csvfile:
        writer = csv.writer(csvfile)
        writer.writerow(["Block_idx", "position_start", "position_end", "most_likely_state"])
        for block_idx, res in enumerate(viterbi_result):
            if len(res) == 0:
                continue
            if ref_coordinates is None:
                seg, cur = 0, res[0]
                for pos in range(1, len(res)):
                    if res[pos] != cur:
                        writer.writerow([block_idx, seg, pos - 1, cur])
                        seg, cur = pos, res[pos]
                writer.writerow([block_idx, seg, len(res) - 1, cur])
            else:
                rc = ref_coordinates[block_idx]
                first = next((i for i, x in enumerate(rc) if x != -9), None)
                if first is None:
                    continue
                seg = rc[first]
                cur_nn = seg
                cur = res[first]
                for pos in range(first, len(res)):
                    if seg == -9:
                        seg = rc[pos]
                        cur = res[pos]
                        cur_nn = seg
                        continue
                    if res[pos] != cur:
                        writer.writerow([block_idx, seg, cur_nn, cur])
                        seg = rc[pos]
                        cur = res[pos]
                    cur_nn = rc[pos] if rc[pos] != -9 else cur_nn
                if not (seg == cur_nn == -9):
                    writer.writerow([block_idx, seg, cur_nn, cur])


def posterior_csv(output_file, posterior_results, ref_coordinates=None):
    with open(output_file, "w", newline="") as csvfile:
        writer = csv.writer(csvfile)
        n_states = posterior_results[0].shape[1] if posterior_results else 0
        writer.writerow(["alignment_block_idx", "position_idx"] +
                        [f"prob_state_{i}" for i in range(n_states)])
        for block_idx, arr in enumerate(posterior_results):
            for pos_idx, row in enumerate(arr):
                if ref_coordinates is None:
                    writer.writerow([block_idx, pos_idx] + row.tolist())
                else:
                    writer.writerow([block_idx, ref_coordinates[block_idx][pos_idx]] + row.tolist())
