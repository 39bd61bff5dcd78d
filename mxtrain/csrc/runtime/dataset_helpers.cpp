// Host-side dataset index builders (native equivalents of the Megatron-DeepSpeed
// `helpers` extension the reference's GPT pre-training pulls in upstream; SURVEY §2.10,
// §2.11 "--data-impl mmap --split 949,50,1").
//
// * mx_build_sample_idx   -- maps every training sample (seq_length+1 tokens drawn from
//                            a concatenated, epoch-shuffled document stream) to
//                            (position in doc_idx, token offset in that document);
// * mx_build_blending_indices -- weighted interleaving of several datasets with the
//                            smallest running deviation from the target weights;
// * mx_count_tokens       -- sum of document sizes over a doc range (split sizing).
//
// Plain C ABI, bound with ctypes from mxtrain/data/gpt_dataset.py.
#include <cstdint>
#include <cstring>
#include <vector>

#define MX_EXPORT extern "C" __attribute__((visibility("default")))

MX_EXPORT int64_t mx_sample_count(int64_t num_epochs, int64_t tokens_per_epoch, int32_t seq_length) {
    // the last token of a sample is the first of the next, so each sample consumes
    // seq_length new tokens and the stream needs one extra token at the end
    return (num_epochs * tokens_per_epoch - 1) / seq_length;
}

MX_EXPORT int mx_build_sample_idx(const int32_t* sizes, const int32_t* doc_idx, int64_t n_doc_idx,
                                  int32_t seq_length, int64_t num_samples, int64_t* out) {
    int64_t di = 0;        // index into doc_idx
    int64_t off = 0;       // token offset inside the current document
    out[0] = 0;
    out[1] = 0;
    for (int64_t s = 1; s <= num_samples; ++s) {
        int64_t remaining = (int64_t)seq_length + 1;
        while (remaining != 0) {
            if (di >= n_doc_idx) return -1;   // ran out of documents: caller sized epochs too small
            const int64_t doc_len = (int64_t)sizes[doc_idx[di]] - off;
            remaining -= doc_len;
            if (remaining <= 0) {
                // sample ends inside this document; the next starts on its last token
                off += remaining + doc_len - 1;
                remaining = 0;
            } else {
                ++di;
                off = 0;
            }
        }
        out[2 * s] = di;
        out[2 * s + 1] = off;
    }
    return 0;
}

MX_EXPORT void mx_build_blending_indices(uint8_t* dataset_index, int64_t* dataset_sample_index,
                                         const double* weights, int32_t num_datasets, int64_t size) {
    std::vector<int64_t> current(num_datasets, 0);
    for (int64_t i = 0; i < size; ++i) {
        const double denom = (double)(i + 1);
        int32_t best = 0;
        double best_err = -1e300;
        for (int32_t d = 0; d < num_datasets; ++d) {
            const double err = weights[d] * denom - (double)current[d];
            if (err > best_err) {
                best_err = err;
                best = d;
            }
        }
        dataset_index[i] = (uint8_t)best;
        dataset_sample_index[i] = current[best];
        ++current[best];
    }
}

MX_EXPORT int64_t mx_count_tokens(const int32_t* sizes, const int64_t* doc_to_seq, int64_t doc_begin,
                                  int64_t doc_end) {
    // doc_to_seq: document index array (length ndocs+1) of sequence boundaries
    int64_t t = 0;
    for (int64_t d = doc_begin; d < doc_end; ++d)
        for (int64_t q = doc_to_seq[d]; q < doc_to_seq[d + 1]; ++q) t += sizes[q];
    return t;
}
