// ingest.cpp -- paired FASTQ(.gz) ingest into the device read layout (SURVEY.md §8 f rank 1:
// the fq1/fq2 inputs that `bwa mem -M -t T anchor fq1 fq2` reads at Anchored_Fusion.py:182).
// Host code only; no GPU call.
//
// Record syntax follows the reader bwa uses (kseq): a record starts at a line beginning with
// '@' (FASTQ) or '>' (FASTA); the name is the header up to the first space or tab, with a
// trailing "/<digit>" removed (bwa's trim_readno); sequence lines run to the '+' line (or to
// the next header for FASTA records); quality lines run until they cover the sequence.  Blank
// lines between records are skipped, '\r' before '\n' is dropped.  As in bwa's paired mode,
// the two files must hold the same number of records with equal names pair by pair.
//
// Layout written by af_fastq_export (include/afgpu.h): pair-major rows of `stride` bytes
// (row 2p = mate 1, row 2p+1 = mate 2), ASCII bases as read, 'N'-padded; lens[2p + m]; the
// QNAMEs of the pairs NUL-terminated in one arena with an offset per pair.
//
// Threads: af_fastq_next parses the two files concurrently (one thread each: zlib inflate +
// line scan with memchr); af_fastq_export copies rows with up to `threads` threads.
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/afgpu.h"

namespace {

// A line source over gzread (zlib reads plain files as they are).
struct Src {
    gzFile gz = nullptr;
    std::string path;
    std::vector<char> buf = std::vector<char>(1 << 22);
    size_t beg = 0, end = 0;
    bool eof = false;
    int64_t line_no = 0;
    std::string pending;  // one pushed-back line
    bool has_pending = false;
    std::string err;

    ~Src() {
        if (gz) gzclose(gz);
    }
    bool open(const char *p) {
        path = p;
        gz = gzopen(p, "rb");
        if (!gz) {
            err = "cannot open " + path;
            return false;
        }
        gzbuffer(gz, 1 << 20);
        return true;
    }
    // Next line as [p, p + n), terminator and a trailing '\r' removed; valid until the next
    // call.  Returns false at the end of input (or on a read error: err is set).
    bool line(const char *&p, size_t &n) {
        if (has_pending) {
            has_pending = false;
            p = pending.data();
            n = pending.size();
            return true;
        }
        for (;;) {
            const char *s = buf.data() + beg;
            const char *nl = static_cast<const char *>(memchr(s, '\n', end - beg));
            if (nl || (eof && beg < end)) {
                p = s;
                n = nl ? (size_t)(nl - s) : end - beg;
                beg = nl ? (size_t)(nl - buf.data()) + 1 : end;
                if (n && p[n - 1] == '\r') --n;
                ++line_no;
                return true;
            }
            if (eof) return false;
            memmove(buf.data(), s, end - beg);
            end -= beg;
            beg = 0;
            if (end == buf.size()) buf.resize(buf.size() * 2);  // a line longer than the buffer
            const int r = gzread(gz, buf.data() + end, (unsigned)std::min<size_t>(buf.size() - end, 1u << 30));
            if (r < 0) {
                int zerr = 0;
                const char *m = gzerror(gz, &zerr);
                err = path + ": read error: " + (m ? m : "?");
                eof = true;
                return false;
            }
            if (r == 0) eof = true;
            end += (size_t)r;
        }
    }
    void push_back(const char *p, size_t n) {
        pending.assign(p, n);
        has_pending = true;
    }
};

// One parsed batch of one file: names and sequences in arenas.
struct Batch {
    std::vector<char> names, seqs;
    std::vector<int64_t> name_off{0}, seq_off{0};
    int64_t n() const { return (int64_t)name_off.size() - 1; }
    void clear() {
        names.clear();
        seqs.clear();
        name_off.assign(1, 0);
        seq_off.assign(1, 0);
    }
};

// Parses up to max_n further records of src into b.  Returns false on malformed input.
bool parse(Src &src, int64_t max_n, Batch &b) {
    b.clear();
    const char *p;
    size_t n;
    while (b.n() < max_n) {
        // header (blank lines skipped)
        bool got = false;
        while (src.line(p, n)) {
            if (n == 0) continue;
            got = true;
            break;
        }
        if (!got) return src.err.empty();
        if (p[0] != '@' && p[0] != '>') {
            src.err = src.path + ":" + std::to_string(src.line_no) + ": expected a '@' or '>' record header";
            return false;
        }
        const bool fastq = p[0] == '@';
        size_t e = 1;
        while (e < n && p[e] != ' ' && p[e] != '\t') ++e;
        size_t nl = e - 1;
        if (nl > 2 && p[e - 2] == '/' && p[e - 1] >= '0' && p[e - 1] <= '9') nl -= 2;  // trim_readno
        b.names.insert(b.names.end(), p + 1, p + 1 + nl);
        b.names.push_back('\0');
        b.name_off.push_back((int64_t)b.names.size());
        // sequence lines
        const size_t s0 = b.seqs.size();
        bool plus = false;
        while (src.line(p, n)) {
            if (n && p[0] == '+' && fastq) {
                plus = true;
                break;
            }
            if (n && (p[0] == '>' || (p[0] == '@' && !fastq))) {  // next record of a FASTA file
                src.push_back(p, n);
                break;
            }
            b.seqs.insert(b.seqs.end(), p, p + n);
        }
        if (!src.err.empty()) return false;
        const size_t slen = b.seqs.size() - s0;
        if (fastq) {
            if (!plus) {
                src.err = src.path + ": truncated FASTQ record (no '+' line)";
                return false;
            }
            size_t ql = 0;
            while (ql < slen && src.line(p, n)) ql += n;
            if (ql < slen) {
                src.err = src.path + ": truncated FASTQ record (quality shorter than sequence)";
                return false;
            }
        }
        b.seq_off.push_back((int64_t)b.seqs.size());
    }
    return true;
}

}  // namespace

struct af_fastq {
    Src src[2];
    Batch bat[2];
    int threads = 1;
    int64_t pairs_done = 0;
    std::string err;
};

extern "C" {

int af_fastq_open(const char *fq1, const char *fq2, int threads, af_fastq **out) {
    if (!out || !fq1 || !fq2) return AF_E_INVALID;
    *out = nullptr;
    af_fastq *f = new (std::nothrow) af_fastq;
    if (!f) return AF_E_NOMEM;
    f->threads = threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (!f->src[0].open(fq1) || !f->src[1].open(fq2)) {
        f->err = f->src[0].err.empty() ? f->src[1].err : f->src[0].err;
        *out = f;  // the handle carries the message; the caller closes it
        return AF_E_INVALID;
    }
    *out = f;
    return AF_OK;
}

const char *af_fastq_error(const af_fastq *f) { return f ? f->err.c_str() : "null af_fastq handle"; }

void af_fastq_close(af_fastq *f) { delete f; }

int af_fastq_next(af_fastq *f, int64_t max_pairs, int64_t *n_pairs, int32_t *max_len, int64_t *names_bytes) {
    if (!f || !n_pairs || max_pairs < 0) return AF_E_INVALID;
    *n_pairs = 0;
    bool ok[2] = {true, true};
    std::thread t([&] { ok[1] = parse(f->src[1], max_pairs, f->bat[1]); });
    ok[0] = parse(f->src[0], max_pairs, f->bat[0]);
    t.join();
    for (int m = 0; m < 2; ++m)
        if (!ok[m]) {
            f->err = f->src[m].err;
            return AF_E_INVALID;
        }
    const Batch &b1 = f->bat[0], &b2 = f->bat[1];
    if (b1.n() != b2.n()) {
        f->err = "paired FASTQs differ in length: " + std::to_string(f->pairs_done + b1.n()) + " vs " +
                 std::to_string(f->pairs_done + b2.n()) + " records";
        return AF_E_INVALID;
    }
    int32_t ml = 0;
    for (int64_t i = 0; i < b1.n(); ++i) {
        const char *a = b1.names.data() + b1.name_off[i], *b = b2.names.data() + b2.name_off[i];
        if (strcmp(a, b) != 0) {  // bwa: "paired reads have different names"
            f->err = std::string("paired reads have different names: \"") + a + "\", \"" + b + "\"";
            return AF_E_INVALID;
        }
        ml = std::max<int32_t>(ml, (int32_t)std::max(b1.seq_off[i + 1] - b1.seq_off[i], b2.seq_off[i + 1] - b2.seq_off[i]));
    }
    f->pairs_done += b1.n();
    *n_pairs = b1.n();
    if (max_len) *max_len = ml;
    if (names_bytes) *names_bytes = (int64_t)b1.names.size();
    return AF_OK;
}

int af_fastq_export(af_fastq *f, int32_t stride, uint8_t *reads, int32_t *lens, char *names, int64_t names_cap,
                    int64_t *name_off) {
    if (!f || stride < 0) return AF_E_INVALID;
    const Batch &b1 = f->bat[0], &b2 = f->bat[1];
    const int64_t n = b1.n();
    if (names && (int64_t)b1.names.size() > names_cap) {
        f->err = "names arena too small";
        return AF_E_CAPACITY;
    }
    for (int64_t i = 0; i < n; ++i)
        if (b1.seq_off[i + 1] - b1.seq_off[i] > stride || b2.seq_off[i + 1] - b2.seq_off[i] > stride) {
            f->err = "read longer than stride " + std::to_string(stride);
            return AF_E_CAPACITY;
        }
    auto rows = [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i)
            for (int m = 0; m < 2; ++m) {
                const Batch &b = f->bat[m];
                const int64_t l = b.seq_off[i + 1] - b.seq_off[i];
                if (reads) {
                    uint8_t *row = reads + (2 * i + m) * (int64_t)stride;
                    memcpy(row, b.seqs.data() + b.seq_off[i], (size_t)l);
                    memset(row + l, 'N', (size_t)(stride - l));
                }
                if (lens) lens[2 * i + m] = (int32_t)l;
            }
    };
    const int T = (int)std::min<int64_t>(f->threads, std::max<int64_t>(1, n / 4096));
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(rows, n * k / T, n * (k + 1) / T);
    rows(0, n / T);
    if (names) memcpy(names, b1.names.data(), b1.names.size());
    if (name_off)
        for (int64_t i = 0; i < n; ++i) name_off[i] = b1.name_off[i];
    for (auto &x : th) x.join();
    return AF_OK;
}

}  // extern "C"
