// post.cpp -- output formats of the post stack (host code behind the C-ABI):
//   cwf_write_vtu        <- cwf::post::write_vtu        (src/post/vtu_writer.cpp:171-297)
//   cwf_probe_log_frame  <- cwf::post::ProbeLogger      (src/post/probe_logger.cpp:21-124)
// Byte-for-byte the reference's files: VTU XML header text and attribute order, raw appended data
// with UInt32 block headers in the reference's block order, Float32 arrays, Int32 connectivity /
// offsets, UInt8 VTK types (10 tet, 12 hex), points = position0 + u in f32; probe CSV rows with
// std::fixed precision 9 (printf "%.9f").
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

namespace cwf
{
namespace
{

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

struct Blob
{
    std::vector<uint8_t> bytes;
    // vtu_writer.cpp:133-147: UInt32 payload size, then the payload; returns the block's offset
    uint64_t append(const void *data, uint64_t n)
    {
        if (n > 0xFFFFFFFFull)
            throw std::runtime_error("VTU block exceeds UInt32 header limit");
        const uint64_t off = bytes.size();
        const uint32_t sz = (uint32_t)n;
        const uint8_t *p = reinterpret_cast<const uint8_t *>(&sz);
        bytes.insert(bytes.end(), p, p + 4);
        const uint8_t *b = reinterpret_cast<const uint8_t *>(data);
        bytes.insert(bytes.end(), b, b + n);
        return off;
    }
};

// field k (0..12) of every 13-float record
std::vector<float> gather_fields(const float *rec, uint64_t count, int first, int comps)
{
    std::vector<float> out(count * comps);
    for (uint64_t i = 0; i < count; ++i)
        for (int c = 0; c < comps; ++c)
            out[i * comps + c] = rec[13 * i + first + c];
    return out;
}

int local_count(const uint32_t *conn, uint64_t e)
{
    int n = 0;
    while (n < 8 && conn[8 * e + n] != kInvalid)
        ++n;
    return n;
}

struct File
{
    FILE *f = nullptr;
    ~File()
    {
        if (f)
            fclose(f);
    }
};

void make_parent(const std::string &path)
{
    const std::filesystem::path p(path);
    if (!p.parent_path().empty())
        std::filesystem::create_directories(p.parent_path());
}

}  // namespace
}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_write_vtu(const char *path, const cwf_frame_view *f, double simulation_time, uint32_t frame_index)
{
    if (!path || !f || !f->position0 || !f->displacement || !f->velocity || !f->acceleration ||
        !f->element_fields || !f->node_fields || (!f->connectivity && f->element_count))
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    try
    {
        make_parent(path);
        File file;
        file.f = fopen(path, "wb");
        if (!file.f)
            return set_error(nullptr, CWF_ERR_IO, "failed to open VTU file", path);
        const uint64_t N = f->node_count, E = f->element_count;
        std::vector<float> points(3 * N);
        for (uint64_t i = 0; i < 3 * N; ++i)
            points[i] = f->position0[i] + f->displacement[i];  // f32, vtu_writer.cpp:53-65
        std::vector<int32_t> conn, offs;
        std::vector<uint8_t> types;
        conn.reserve(E * 8);
        offs.reserve(E);
        types.reserve(E);
        int32_t running = 0;
        for (uint64_t e = 0; e < E; ++e)  // vtu_writer.cpp:106-131: tet4 -> 4 nodes / VTK 10, else 8 / VTK 12
        {
            const int lc = local_count(f->connectivity, e) == 4 ? 4 : 8;
            for (int a = 0; a < lc; ++a)
                conn.push_back((int32_t)f->connectivity[8 * e + a]);
            running += lc;
            offs.push_back(running);
            types.push_back(lc == 4 ? 10 : 12);
        }
        Blob blob;
        blob.bytes.reserve(4 * (6 * N) + 64);
        uint64_t po[6], co[3];
        po[0] = blob.append(f->displacement, 12 * N);
        po[1] = blob.append(f->velocity, 12 * N);
        po[2] = blob.append(f->acceleration, 12 * N);
        {
            const auto s = gather_fields(f->node_fields, N, 0, 6);
            po[3] = blob.append(s.data(), 4 * s.size());
            const auto t = gather_fields(f->node_fields, N, 6, 6);
            po[4] = blob.append(t.data(), 4 * t.size());
            const auto v = gather_fields(f->node_fields, N, 12, 1);
            po[5] = blob.append(v.data(), 4 * v.size());
        }
        {
            const auto s = gather_fields(f->element_fields, E, 0, 6);
            co[0] = blob.append(s.data(), 4 * s.size());
            const auto t = gather_fields(f->element_fields, E, 6, 6);
            co[1] = blob.append(t.data(), 4 * t.size());
            const auto v = gather_fields(f->element_fields, E, 12, 1);
            co[2] = blob.append(v.data(), 4 * v.size());
        }
        const uint64_t pts_off = blob.append(points.data(), 4 * points.size());
        const uint64_t conn_off = blob.append(conn.data(), 4 * conn.size());
        const uint64_t offs_off = blob.append(offs.data(), 4 * offs.size());
        const uint64_t types_off = blob.append(types.data(), types.size());

        FILE *o = file.f;
        fprintf(o, "<?xml version=\"1.0\"?>\n");
        fprintf(o, "<VTKFile type=\"UnstructuredGrid\" version=\"1.0\" byte_order=\"LittleEndian\" "
                   "header_type=\"UInt32\">\n");
        fprintf(o, "  <UnstructuredGrid>\n");
        fprintf(o, "    <FieldData>\n");
        // std::ostream << double: defaultfloat, precision 6 == "%g"
        fprintf(o, "      <DataArray type=\"Float64\" Name=\"time\" NumberOfTuples=\"1\">%g</DataArray>\n",
                simulation_time);
        fprintf(o, "      <DataArray type=\"UInt32\" Name=\"frame\" NumberOfTuples=\"1\">%" PRIu32 "</DataArray>\n",
                frame_index);
        fprintf(o, "    </FieldData>\n");
        fprintf(o, "    <Piece NumberOfPoints=\"%" PRIu64 "\" NumberOfCells=\"%" PRIu64 "\">\n", N, E);
        static const char *pn[6] = {"displacement", "velocity", "acceleration", "strain_node", "stress_node",
                                    "von_mises_node"};
        static const int pc[6] = {3, 3, 3, 6, 6, 1};
        fprintf(o, "      <PointData Scalars=\"von_mises_node\">\n");
        for (int i = 0; i < 6; ++i)
            fprintf(o,
                    "        <DataArray type=\"Float32\" Name=\"%s\" NumberOfComponents=\"%d\" format=\"appended\" "
                    "offset=\"%" PRIu64 "\"/>\n",
                    pn[i], pc[i], po[i]);
        fprintf(o, "      </PointData>\n");
        static const char *cn[3] = {"strain_elem", "stress_elem", "von_mises_elem"};
        static const int cc[3] = {6, 6, 1};
        fprintf(o, "      <CellData Scalars=\"von_mises_elem\">\n");
        for (int i = 0; i < 3; ++i)
            fprintf(o,
                    "        <DataArray type=\"Float32\" Name=\"%s\" NumberOfComponents=\"%d\" format=\"appended\" "
                    "offset=\"%" PRIu64 "\"/>\n",
                    cn[i], cc[i], co[i]);
        fprintf(o, "      </CellData>\n");
        fprintf(o, "      <Points>\n");
        fprintf(o,
                "        <DataArray type=\"Float32\" NumberOfComponents=\"3\" format=\"appended\" offset=\"%" PRIu64
                "\"/>\n",
                pts_off);
        fprintf(o, "      </Points>\n");
        fprintf(o, "      <Cells>\n");
        fprintf(o,
                "        <DataArray type=\"Int32\" Name=\"connectivity\" format=\"appended\" offset=\"%" PRIu64
                "\"/>\n",
                conn_off);
        fprintf(o, "        <DataArray type=\"Int32\" Name=\"offsets\" format=\"appended\" offset=\"%" PRIu64 "\"/>\n",
                offs_off);
        fprintf(o, "        <DataArray type=\"UInt8\" Name=\"types\" format=\"appended\" offset=\"%" PRIu64 "\"/>\n",
                types_off);
        fprintf(o, "      </Cells>\n");
        fprintf(o, "    </Piece>\n");
        fprintf(o, "  </UnstructuredGrid>\n");
        fprintf(o, "  <AppendedData encoding=\"raw\">\n");
        fputc('_', o);
        if (!blob.bytes.empty() && fwrite(blob.bytes.data(), 1, blob.bytes.size(), o) != blob.bytes.size())
            return set_error(nullptr, CWF_ERR_IO, "failed to write VTU payload", path);
        fprintf(o, "\n  </AppendedData>\n");
        fprintf(o, "</VTKFile>\n");
        if (fflush(o) != 0)
            return set_error(nullptr, CWF_ERR_IO, "failed to write VTU file", path);
        return 0;
    }
    catch (const std::exception &ex)
    {
        return set_error(nullptr, CWF_ERR_IO, ex.what(), path);
    }
}

int cwf_probe_log_frame(const char *path, int *header_written, const uint32_t *probes, uint64_t probe_count,
                        const cwf_frame_view *f, double simulation_time, uint32_t frame_index)
{
    if (!path || !header_written || (probe_count && (!probes || !f)))
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (probe_count == 0)  // probe_logger.cpp:99-103
        return 0;
    try
    {
        if (!*header_written)  // write_header (probe_logger.cpp:64-89): truncate + header row
        {
            make_parent(path);
            File hf;
            hf.f = fopen(path, "w");
            if (!hf.f)
                return set_error(nullptr, CWF_ERR_IO, "failed to open probe CSV for header", path);
            fputs("frame,time,node,ux,uy,uz,vx,vy,vz,ax,ay,az"
                  ",strain_xx,strain_yy,strain_zz,strain_xy,strain_yz,strain_xz"
                  ",stress_xx,stress_yy,stress_zz,stress_xy,stress_yz,stress_xz,von_mises\n",
                  hf.f);
            *header_written = 1;
        }
        File file;
        file.f = fopen(path, "a");
        if (!file.f)
            return set_error(nullptr, CWF_ERR_IO, "failed to open probe CSV", path);
        for (uint64_t i = 0; i < probe_count; ++i)
        {
            const uint32_t n = probes[i];
            if (n >= f->node_count)
                return set_error(nullptr, CWF_ERR_INDEX, "probe index out of range", std::to_string(n));
            // serialize_row (probe_logger.cpp:21-55): std::fixed, precision 9
            fprintf(file.f, "%" PRIu32 ",%.9f,%" PRIu32, frame_index, simulation_time, n);
            const float *kin[3] = {f->displacement, f->velocity, f->acceleration};
            for (const float *k : kin)
                for (int c = 0; c < 3; ++c)
                    fprintf(file.f, ",%.9f", (double)k[3ull * n + c]);
            const float *nf = f->node_fields + 13ull * n;
            for (int c = 0; c < 13; ++c)
                fprintf(file.f, ",%.9f", (double)nf[c]);
            fputc('\n', file.f);
        }
        return 0;
    }
    catch (const std::exception &ex)
    {
        return set_error(nullptr, CWF_ERR_IO, ex.what(), path);
    }
}

}  // extern "C"
