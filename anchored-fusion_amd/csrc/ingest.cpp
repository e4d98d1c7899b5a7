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
// line scan with memchr, the decompression running ahead on a reader thread of its own, up to
// three 8 MiB chunks in flight); af_fastq_export copies rows with up to `threads` threads.  BGZF
// input (blocked gzip, as bgzip/htslib write it: each member carries its compressed size in a
// "BC" extra field) is inflated block-parallel: batches of up to 512 blocks, threads/2 per
// file, each block checked against its CRC32.
#include <zlib.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <exception>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/afgpu.h"

namespace {

// A line source over gzread (zlib reads plain files as they are).
struct Src {
    gzFile gz = nullptr;
    FILE *fp = nullptr;            // BGZF input (read raw, inflated block-parallel)
    int n_threads = 1;
    std::vector<char> dec;         // BGZF: inflated bytes not yet handed to `buf`
    size_t dec_pos = 0;
    bool bgzf_eof = false;
    std::string path;
    std::vector<char> buf = std::vector<char>(1 << 22);
    size_t beg = 0, end = 0;
    bool eof = false;
    int64_t line_no = 0;
    std::string pending;  // one pushed-back line
    bool has_pending = false;
    std::string err;
    // reader thread: decompressed chunks queued ahead of the line scan
    std::thread reader;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::vector<char>> chunks;
    size_t chunk_pos = 0;
    bool r_done = false, r_error = false, r_stop = false;

    ~Src() {
        if (reader.joinable()) {
            {
                std::lock_guard<std::mutex> g(mu);
                r_stop = true;
            }
            cv.notify_all();
            reader.join();
        }
        if (gz) gzclose(gz);
        if (fp) fclose(fp);
    }
    void start_reader() {
        reader = std::thread([this] {
            for (;;) {
                std::vector<char> c;
                long r;
                try {  // no exception may leave the thread (std::terminate): report it as a read error
                    c.resize(8u << 20);
                    r = read_some(c.data(), c.size());
                } catch (const std::exception &ex) {
                    err = path + ": " + ex.what();
                    r = -1;
                }
                std::unique_lock<std::mutex> g(mu);
                if (r <= 0) {
                    r_error = r < 0;
                    r_done = true;
                    cv.notify_all();
                    return;
                }
                c.resize((size_t)r);
                chunks.push_back(std::move(c));
                cv.notify_all();
                cv.wait(g, [this] { return chunks.size() < 3 || r_stop; });
                if (r_stop) return;
            }
        });
    }
    // the next decompressed bytes from the reader thread (0 at the end, -1 on error)
    long pull(char *dst, size_t cap) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [this] { return !chunks.empty() || r_done; });
        if (chunks.empty()) return r_error ? -1 : 0;
        std::vector<char> &c = chunks.front();
        const size_t k = std::min(cap, c.size() - chunk_pos);
        memcpy(dst, c.data() + chunk_pos, k);
        chunk_pos += k;
        if (chunk_pos == c.size()) {
            chunks.pop_front();
            chunk_pos = 0;
            cv.notify_all();
        }
        return (long)k;
    }
    // block size of the BGZF member whose 12-byte fixed header + extra field is at h (or -1)
    static long bgzf_bsize(const unsigned char *h, size_t n) {
        if (n < 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return -1;
        const size_t xlen = h[10] | (h[11] << 8);
        for (size_t o = 12; o + 4 <= 12 + xlen && o + 4 <= n;) {
            const size_t slen = h[o + 2] | (h[o + 3] << 8);
            if (h[o] == 66 && h[o + 1] == 67 && slen == 2 && o + 6 <= n) return (long)(h[o + 4] | (h[o + 5] << 8)) + 1;
            o += 4 + slen;
        }
        return -1;
    }
    bool open(const char *p, int threads) {
        path = p;
        n_threads = threads > 0 ? threads : 1;
        if (FILE *f = fopen(p, "rb")) {  // BGZF?  (the first member has the BC field)
            unsigned char h[64];
            const size_t n = fread(h, 1, sizeof h, f);
            if (bgzf_bsize(h, n) > 0) {
                rewind(f);
                fp = f;
                start_reader();
                return true;
            }
            fclose(f);
        }
        gz = gzopen(p, "rb");
        if (!gz) {
            err = "cannot open " + path;
            return false;
        }
        gzbuffer(gz, 1 << 20);
        char c0;  // plain text reads as fast as it is scanned: no reader thread for it
        if (gzread(gz, &c0, 0) >= 0 && !gzdirect(gz)) start_reader();
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
            const size_t cap = std::min<size_t>(buf.size() - end, 1u << 30);
            const long r = reader.joinable() ? pull(buf.data() + end, cap) : read_some(buf.data() + end, cap);
            if (r < 0) {
                eof = true;
                return false;
            }
            if (r == 0) eof = true;
            end += (size_t)r;
        }
    }
    // up to cap decompressed bytes into dst; 0 at the end of input, -1 on error (err set)
    long read_some(char *dst, size_t cap) {
        if (!fp) {
            const int r = gzread(gz, dst, (unsigned)cap);
            if (r < 0) {
                int zerr = 0;
                const char *m = gzerror(gz, &zerr);
                err = path + ": read error: " + (m ? m : "?");
            }
            return r;
        }
        while (dec_pos == dec.size() && !bgzf_eof)  // (a batch may hold only empty blocks)
            if (!bgzf_batch()) return -1;
        const size_t k = std::min(cap, dec.size() - dec_pos);
        memcpy(dst, dec.data() + dec_pos, k);
        dec_pos += k;
        return (long)k;
    }
    // reads up to 512 BGZF blocks and inflates them in parallel into `dec`
    bool bgzf_batch() {
        std::vector<std::vector<unsigned char>> blocks;
        std::vector<size_t> out_off{0};
        while (blocks.size() < 512) {
            unsigned char h[18];
            const size_t n = fread(h, 1, 12, fp);
            if (n == 0) {
                bgzf_eof = true;
                break;
            }
            if (n < 12) return fail_bgzf("truncated BGZF block header");
            const size_t xlen = h[10] | (h[11] << 8);
            std::vector<unsigned char> b(12 + xlen);
            memcpy(b.data(), h, 12);
            if (fread(b.data() + 12, 1, xlen, fp) != xlen) return fail_bgzf("truncated BGZF extra field");
            const long bsize = bgzf_bsize(b.data(), b.size());
            if (bsize < (long)(12 + xlen + 8)) return fail_bgzf("gzip member without a BGZF size (mixed input?)");
            b.resize((size_t)bsize);
            if (fread(b.data() + 12 + xlen, 1, (size_t)bsize - 12 - xlen, fp) != (size_t)bsize - 12 - xlen)
                return fail_bgzf("truncated BGZF block");
            const unsigned char *t = b.data() + bsize - 4;
            const size_t isize = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
            if (isize > 65536) return fail_bgzf("corrupt BGZF block (ISIZE above the 64 KiB BGZF maximum)");
            out_off.push_back(out_off.back() + isize);
            blocks.push_back(std::move(b));
        }
        dec.assign(out_off.back(), 0);
        dec_pos = 0;
        std::vector<int> bad(blocks.size(), 0);
        auto work = [&](size_t t0, size_t step) {
            for (size_t i = t0; i < blocks.size(); i += step) {
                const std::vector<unsigned char> &b = blocks[i];
                const size_t xlen = b[10] | (b[11] << 8), cstart = 12 + xlen, clen = b.size() - cstart - 8;
                const size_t isize = out_off[i + 1] - out_off[i];
                z_stream z{};
                if (inflateInit2(&z, -15) != Z_OK) { bad[i] = 1; continue; }
                z.next_in = const_cast<unsigned char *>(b.data() + cstart);
                z.avail_in = (uInt)clen;
                unsigned char spare;  // an empty block (the EOF marker): zlib needs a non-null output
                z.next_out = isize ? reinterpret_cast<unsigned char *>(dec.data() + out_off[i]) : &spare;
                z.avail_out = isize ? (uInt)isize : 1u;
                const int rc = inflate(&z, Z_FINISH);
                inflateEnd(&z);
                const unsigned char *c = b.data() + b.size() - 8;
                const uLong crc = (uLong)c[0] | ((uLong)c[1] << 8) | ((uLong)c[2] << 16) | ((uLong)c[3] << 24);
                if (rc != Z_STREAM_END || z.total_out != isize ||
                    crc32(0L, reinterpret_cast<const Bytef *>(dec.data() + out_off[i]), (uInt)isize) != crc)
                    bad[i] = 1;
            }
        };
        const size_t T = std::min<size_t>((size_t)n_threads, std::max<size_t>(1, blocks.size()));
        std::vector<std::thread> th;
        for (size_t k = 1; k < T; ++k) th.emplace_back(work, k, T);
        work(0, T);
        for (auto &x : th) x.join();
        for (size_t i = 0; i < blocks.size(); ++i)
            if (bad[i]) return fail_bgzf("corrupt BGZF block (inflate or CRC32)");
        return true;
    }
    bool fail_bgzf(const char *what) {
        err = path + ": " + what;
        return false;
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


// ---- sharded ingest: the records of one part of one BGZF file ---------------------------------
// Part p of P takes the BGZF blocks whose compressed offset lies in [p S / P, (p + 1) S / P)
// (S = file size) and owns the FASTQ records whose header starts in their inflated bytes.  Part
// 0 starts at a record; a later part syncs on the first line that opens a 4-line record ('@'
// header, a sequence line, a '+' line, a quality line as long as the sequence, then a header or
// the end).  A record that runs past the part's blocks is completed from the following blocks
// (read ahead, doubled until it fits).  Record syntax as `parse` (FASTQ only).

struct BgzfBlock {
    int64_t off;
    int64_t bsize, isize;
};

bool bgzf_index(FILE *fp, std::vector<BgzfBlock> &blk, std::string &err) {
    if (fseeko(fp, 0, SEEK_END) != 0) { err = "seek failed"; return false; }
    const int64_t size = ftello(fp);
    int64_t off = 0;
    while (off < size) {
        unsigned char h[64];
        if (fseeko(fp, off, SEEK_SET) != 0) { err = "seek failed"; return false; }
        const size_t n = fread(h, 1, sizeof h, fp);
        const long bsize = Src::bgzf_bsize(h, n);
        if (bsize < 26 || off + bsize > size) { err = "not a BGZF file (or a truncated block)"; return false; }
        unsigned char t[4];
        if (fseeko(fp, off + bsize - 4, SEEK_SET) != 0 || fread(t, 1, 4, fp) != 4) { err = "truncated BGZF block"; return false; }
        const int64_t isize = (int64_t)t[0] | ((int64_t)t[1] << 8) | ((int64_t)t[2] << 16) | ((int64_t)t[3] << 24);
        if (isize > 65536) { err = "corrupt BGZF block (ISIZE above 64 KiB)"; return false; }
        blk.push_back(BgzfBlock{off, bsize, isize});
        off += bsize;
    }
    return true;
}

// blocks [b0, b1) inflated (block-parallel, CRC-checked) into out
bool bgzf_inflate(FILE *fp, const std::vector<BgzfBlock> &blk, size_t b0, size_t b1, int threads, std::vector<char> &out,
                  std::string &err) {
    out.clear();
    if (b0 >= b1) return true;
    const int64_t c0 = blk[b0].off, c1 = blk[b1 - 1].off + blk[b1 - 1].bsize;
    std::vector<unsigned char> comp((size_t)(c1 - c0));
    if (fseeko(fp, c0, SEEK_SET) != 0 || fread(comp.data(), 1, comp.size(), fp) != comp.size()) {
        err = "read error";
        return false;
    }
    std::vector<int64_t> o(b1 - b0 + 1, 0);
    for (size_t i = b0; i < b1; ++i) o[i - b0 + 1] = o[i - b0] + blk[i].isize;
    out.assign((size_t)o.back(), 0);
    std::vector<int> bad(b1 - b0, 0);
    auto work = [&](size_t t0, size_t step) {
        for (size_t i = t0; i < b1 - b0; i += step) {
            const BgzfBlock &B = blk[b0 + i];
            const unsigned char *b = comp.data() + (B.off - c0);
            const size_t xlen = b[10] | (b[11] << 8), cstart = 12 + xlen, clen = (size_t)B.bsize - cstart - 8;
            z_stream z{};
            if (inflateInit2(&z, -15) != Z_OK) { bad[i] = 1; continue; }
            z.next_in = const_cast<unsigned char *>(b + cstart);
            z.avail_in = (uInt)clen;
            unsigned char spare;  // an empty block (the EOF marker) still needs room to finish
            z.next_out = B.isize ? reinterpret_cast<unsigned char *>(out.data() + o[i]) : &spare;
            z.avail_out = B.isize ? (uInt)B.isize : 1u;
            const int rc = inflate(&z, Z_FINISH);
            inflateEnd(&z);
            const unsigned char *c = b + B.bsize - 8;
            const uLong crc = (uLong)c[0] | ((uLong)c[1] << 8) | ((uLong)c[2] << 16) | ((uLong)c[3] << 24);
            if (rc != Z_STREAM_END || (int64_t)z.total_out != B.isize ||
                crc32(0L, reinterpret_cast<const Bytef *>(out.data() + o[i]), (uInt)B.isize) != crc)
                bad[i] = 1;
        }
    };
    const size_t T = std::min<size_t>((size_t)std::max(1, threads), b1 - b0);
    std::vector<std::thread> th;
    for (size_t k = 1; k < T; ++k) th.emplace_back(work, k, T);
    work(0, T);
    for (auto &x : th) x.join();
    for (int v : bad)
        if (v) { err = "corrupt BGZF block (inflate or CRC32)"; return false; }
    return true;
}

// the lines of D from pos: [s, e) without the terminator ('\r' dropped); false at the end
struct MemLines {
    const char *d;
    size_t n, pos = 0;
    bool next(size_t &s, size_t &e) {
        if (pos >= n) return false;
        const char *nl = static_cast<const char *>(memchr(d + pos, '\n', n - pos));
        s = pos;
        e = nl ? (size_t)(nl - d) : n;
        pos = nl ? e + 1 : n;
        if (e > s && d[e - 1] == '\r') --e;
        return true;
    }
};

bool seq_line(const char *p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const char c = p[i];
        if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '.' || c == '-' || c == '*')) return false;
    }
    return true;
}

// the first record start at or after line start `from` (4-line check); n if none
size_t fastq_sync(const std::vector<char> &D, size_t from) {
    const char *d = D.data();
    const size_t n = D.size();
    size_t p = from;
    while (p < n) {
        MemLines L{d, n, p};
        size_t s[5], e[5];
        int got = 0;
        while (got < 5 && L.next(s[got], e[got])) ++got;
        if (got >= 4 && e[0] > s[0] && d[s[0]] == '@' && seq_line(d + s[1], e[1] - s[1]) && e[2] > s[2] &&
            d[s[2]] == '+' && e[3] - s[3] == e[1] - s[1] && (got < 5 || (e[4] > s[4] && d[s[4]] == '@')))
            return p;
        const char *nl = static_cast<const char *>(memchr(d + p, '\n', n - p));
        if (!nl) break;
        p = (size_t)(nl - d) + 1;
    }
    return n;
}

// records with a header at [start, lim) of D into b.  1 = done, 0 = a record runs past the end
// of D (read more), -1 = malformed (err set).  *multi_line: a record's sequence or quality spans
// several lines (kseq accepts it; a part boundary cannot be found by the 4-line rule then)
int parse_mem(const std::vector<char> &D, size_t start, size_t lim, bool at_eof, Batch &b, std::string &err,
              bool *multi_line) {
    b.clear();
    MemLines L{D.data(), D.size(), start};
    const char *d = D.data();
    for (;;) {
        size_t s, e;
        size_t hdr;
        for (;;) {  // header (blank lines skipped)
            hdr = L.pos;
            if (hdr >= lim || !L.next(s, e)) return 1;
            if (e > s) break;
        }
        if (d[s] != '@') { err = "sharded ingest: expected a FASTQ '@' header"; return -1; }
        size_t x = s + 1;
        while (x < e && d[x] != ' ' && d[x] != '\t') ++x;
        size_t nl = x - s - 1;
        if (nl > 2 && d[x - 2] == '/' && d[x - 1] >= '0' && d[x - 1] <= '9') nl -= 2;  // trim_readno
        const size_t name0 = b.names.size(), seq0 = b.seqs.size();
        b.names.insert(b.names.end(), d + s + 1, d + s + 1 + nl);
        b.names.push_back('\0');
        bool plus = false;
        int seq_lines = 0, qual_lines = 0;
        while (L.next(s, e)) {
            if (e > s && d[s] == '+') { plus = true; break; }
            b.seqs.insert(b.seqs.end(), d + s, d + e);
            ++seq_lines;
        }
        const size_t slen = b.seqs.size() - seq0;
        size_t ql = 0;
        while (plus && ql < slen && L.next(s, e)) { ql += e - s; ++qual_lines; }
        if (seq_lines > 1 || qual_lines > 1) *multi_line = true;
        if (!plus || ql < slen) {
            if (!at_eof) {  // the record continues in the next blocks
                b.names.resize(name0);
                b.seqs.resize(seq0);
                return 0;
            }
            err = "truncated FASTQ record";
            return -1;
        }
        b.name_off.push_back((int64_t)b.names.size());
        b.seq_off.push_back((int64_t)b.seqs.size());
        (void)hdr;
    }
}

}  // namespace

struct af_fastq_part {
    Batch b;
    int threads = 1;
    std::string err;
};

static int af_fastq_part_read_impl(const char *path, int part, int parts, int threads, af_fastq_part **out,
                                   int64_t *n_records, int32_t *max_len, int64_t *names_bytes) {
    if (!path || !out || parts < 1 || part < 0 || part >= parts) return AF_E_INVALID;
    af_fastq_part *f = new (std::nothrow) af_fastq_part;
    if (!f) return AF_E_NOMEM;
    *out = f;
    f->threads = threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    FILE *fp = fopen(path, "rb");
    if (!fp) { f->err = std::string("cannot open ") + path; return AF_E_INVALID; }
    std::vector<BgzfBlock> blk;
    bool ok = bgzf_index(fp, blk, f->err);
    if (!ok) {
        fclose(fp);
        f->err = std::string(path) + ": " + f->err;
        return AF_E_UNSUPPORTED;
    }
    const int64_t size = blk.empty() ? 0 : blk.back().off + blk.back().bsize;
    const int64_t lo = size * part / parts, hi = size * (part + 1) / parts;
    size_t b0 = 0, b1 = 0;
    while (b0 < blk.size() && blk[b0].off < lo) ++b0;
    b1 = b0;
    while (b1 < blk.size() && blk[b1].off < hi) ++b1;
    size_t lim = 0;
    for (size_t i = b0; i < b1; ++i) lim += (size_t)blk[i].isize;
    std::vector<char> D;
    int rc = 1;
    bool multi_line = false;
    for (size_t ra = 8;; ra *= 2) {
        const size_t be = std::min(blk.size(), b1 + ra);
        if (!bgzf_inflate(fp, blk, b0, be, f->threads, D, f->err)) { rc = -1; break; }
        const size_t start = part == 0 ? 0 : fastq_sync(D, 0);
        // a 4-line FASTQ reaches its first record start within 4 line ends of any byte; more
        // means records of several lines, which the part rule cannot split
        int lines = 0;
        for (const char *q = D.data(), *qe = D.data() + std::min(start, D.size()); lines <= 4 && q < qe; ++lines) {
            q = static_cast<const char *>(memchr(q, '\n', (size_t)(qe - q)));
            if (!q) break;
            ++q;
        }
        if (lines > 4) { multi_line = true; rc = 1; break; }
        if (start >= lim) { f->b.clear(); rc = 1; break; }  // no record starts in this part
        rc = parse_mem(D, start, lim, be == blk.size(), f->b, f->err, &multi_line);
        if (rc != 0) break;
    }
    fclose(fp);
    if (rc >= 0 && multi_line) {
        f->b.clear();
        f->err = std::string(path) + ": FASTQ records span several lines; parts need 4-line records (read the file whole)";
        return AF_E_UNSUPPORTED;
    }
    if (rc < 0) {
        f->err = std::string(path) + ": " + f->err;
        return AF_E_INVALID;
    }
    int32_t ml = 0;
    for (int64_t i = 0; i < f->b.n(); ++i) ml = std::max<int32_t>(ml, (int32_t)(f->b.seq_off[i + 1] - f->b.seq_off[i]));
    if (n_records) *n_records = f->b.n();
    if (max_len) *max_len = ml;
    if (names_bytes) *names_bytes = (int64_t)f->b.names.size();
    return AF_OK;
}

static int af_fastq_part_export_impl(af_fastq_part *f, int32_t stride, uint8_t *seqs, int32_t *lens, char *names,
                                     int64_t names_cap, int64_t *name_off) {
    if (!f || stride < 0) return AF_E_INVALID;
    const Batch &b = f->b;
    const int64_t n = b.n();
    if (names && (int64_t)b.names.size() > names_cap) { f->err = "names arena too small"; return AF_E_CAPACITY; }
    for (int64_t i = 0; i < n; ++i) {
        const int64_t l = b.seq_off[i + 1] - b.seq_off[i];
        if (l > stride) { f->err = "read longer than stride " + std::to_string(stride); return AF_E_CAPACITY; }
        if (seqs) {
            uint8_t *row = seqs + i * (int64_t)stride;
            memcpy(row, b.seqs.data() + b.seq_off[i], (size_t)l);
            memset(row + l, 'N', (size_t)(stride - l));
        }
        if (lens) lens[i] = (int32_t)l;
        if (name_off) name_off[i] = b.name_off[i];
    }
    if (names) memcpy(names, b.names.data(), b.names.size());
    return AF_OK;
}

struct af_fastq {
    Src src[2];
    Batch bat[2];
    int threads = 1;
    int64_t pairs_done = 0;
    std::string err;
};

static int af_fastq_open_impl(const char *fq1, const char *fq2, int threads, af_fastq **out) {
    if (!out || !fq1 || !fq2) return AF_E_INVALID;
    *out = nullptr;
    af_fastq *f = new (std::nothrow) af_fastq;
    if (!f) return AF_E_NOMEM;
    f->threads = threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int per_file = std::max(1, f->threads / 2);
    if (!f->src[0].open(fq1, per_file) || !f->src[1].open(fq2, per_file)) {
        f->err = f->src[0].err.empty() ? f->src[1].err : f->src[0].err;
        *out = f;  // the handle carries the message; the caller closes it
        return AF_E_INVALID;
    }
    *out = f;
    return AF_OK;
}

const char *af_fastq_error(const af_fastq *f) { return f ? f->err.c_str() : "null af_fastq handle"; }

void af_fastq_close(af_fastq *f) { delete f; }

static int af_fastq_next_impl(af_fastq *f, int64_t max_pairs, int64_t *n_pairs, int32_t *max_len, int64_t *names_bytes) {
    if (!f || !n_pairs || max_pairs < 0) return AF_E_INVALID;
    *n_pairs = 0;
    bool ok[2] = {true, true};
    std::thread t([&] {
        try {  // an exception may not leave the thread
            ok[1] = parse(f->src[1], max_pairs, f->bat[1]);
        } catch (const std::exception &ex) {
            f->src[1].err = ex.what();
            ok[1] = false;
        }
    });
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

static int af_fastq_export_impl(af_fastq *f, int32_t stride, uint8_t *reads, int32_t *lens, char *names, int64_t names_cap,
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

// No C++ exception crosses the C-ABI: allocation failures and anything else thrown below become
// AF_E_* codes (the message goes to af_fastq_error when a handle exists).
template <class F>
static int af_guard(af_fastq *f, F &&body) {
    try {
        return body();
    } catch (const std::bad_alloc &) {
        if (f) f->err = "out of host memory";
        return AF_E_NOMEM;
    } catch (const std::exception &ex) {
        if (f) f->err = ex.what();
        return AF_E_INVALID;
    }
}

extern "C" {

int af_fastq_open(const char *fq1, const char *fq2, int threads, af_fastq **out) {
    try {
        return af_fastq_open_impl(fq1, fq2, threads, out);
    } catch (const std::bad_alloc &) {
        return AF_E_NOMEM;
    } catch (const std::exception &) {
        return AF_E_INVALID;
    }
}

int af_fastq_next(af_fastq *f, int64_t max_pairs, int64_t *n_pairs, int32_t *max_len, int64_t *names_bytes) {
    return af_guard(f, [&] { return af_fastq_next_impl(f, max_pairs, n_pairs, max_len, names_bytes); });
}

int af_fastq_export(af_fastq *f, int32_t stride, uint8_t *reads, int32_t *lens, char *names, int64_t names_cap,
                    int64_t *name_off) {
    return af_guard(f, [&] { return af_fastq_export_impl(f, stride, reads, lens, names, names_cap, name_off); });
}

int af_fastq_part_read(const char *path, int part, int parts, int threads, af_fastq_part **out, int64_t *n_records,
                       int32_t *max_len, int64_t *names_bytes) {
    try {
        return af_fastq_part_read_impl(path, part, parts, threads, out, n_records, max_len, names_bytes);
    } catch (const std::bad_alloc &) {
        if (out && *out) (*out)->err = "out of host memory";
        return AF_E_NOMEM;
    } catch (const std::exception &ex) {
        if (out && *out) (*out)->err = ex.what();
        return AF_E_INVALID;
    }
}

int af_fastq_part_export(af_fastq_part *f, int32_t stride, uint8_t *seqs, int32_t *lens, char *names, int64_t names_cap,
                         int64_t *name_off) {
    try {
        return af_fastq_part_export_impl(f, stride, seqs, lens, names, names_cap, name_off);
    } catch (const std::exception &ex) {
        if (f) f->err = ex.what();
        return AF_E_INVALID;
    }
}

const char *af_fastq_part_error(const af_fastq_part *f) { return f ? f->err.c_str() : "null af_fastq_part handle"; }

void af_fastq_part_free(af_fastq_part *f) { delete f; }

}  // extern "C"
