// gpu_pagereader.go — the in-package half of the MI355X decode path for
// github.com/fraugster/parquet-go (package goparquet).
//
// pageReader / valuesDecoder / levelDecoder are unexported (interfaces.go:11-39,
// hybrid_decoder.go:16-27), so only a file inside package goparquet can stand
// behind them. Copy this file next to chunk_reader.go and apply the three-line
// hook of INTEGRATION.md (a `gpu` field on FileReader / fileReaderOptions and a
// call at the top of readRowGroupData). With WithGPUDecoder(ctx) a FileReader
// decodes each row group's selected column chunks on the GPU in one batch
// (every page, levels and values) and hands ColumnStore.readNextPage
// (data_store.go:236-260) one gpuPageReader per data page, exactly the
// (values, dLevel, rLevel) triple the CPU pageReaders return: the pages before
// a failing page decode normally and the failing page returns its error.
package goparquet

import (
	"context"
	"encoding/binary"
	"fmt"
	"io"
	"math"
	"math/bits"

	"github.com/fraugster/parquet-go/gpudecode"
	"github.com/fraugster/parquet-go/parquet"
)

// WithGPUDecoder routes column-chunk decoding through the MI355X decoder
// bound to ctx (one context per GPU; the FileReader is not goroutine safe,
// file_reader.go:18).
func WithGPUDecoder(ctx *gpudecode.Context) FileReaderOption {
	return func(opts *fileReaderOptions) error {
		opts.gpu = ctx
		return nil
	}
}

// gpuPageReader is one decoded data page (pageReader, interfaces.go:11-18).
type gpuPageReader struct {
	values         []interface{}
	dLevel, rLevel *packedArray
	n              int32
	err            error
}

func (p *gpuPageReader) init(dDecoder, rDecoder getLevelDecoder, values getValueDecoderFn) error {
	return nil
}

func (p *gpuPageReader) read(r io.Reader, ph *parquet.PageHeader, codec parquet.CompressionCodec, validateCRC bool) error {
	return nil
}

func (p *gpuPageReader) numValues() int32 { return p.n }

// readValues returns the whole page (ColumnStore.readNextPage asks for numValues()).
func (p *gpuPageReader) readValues(size int) ([]interface{}, *packedArray, *packedArray, error) {
	if p.err != nil {
		return nil, nil, nil, p.err
	}
	return p.values, p.dLevel, p.rLevel, nil
}

// gpuChunkInput reads one column chunk's bytes and describes it for the decoder (the part of
// readChunk, chunk_reader.go:299-362, before readPages).
func (f *FileReader) gpuChunkInput(col *Column, chunk *parquet.ColumnChunk) ([]byte, gpudecode.ColumnInfo, gpudecode.ChunkMeta, error) {
	var ci gpudecode.ColumnInfo
	var cm gpudecode.ChunkMeta
	if chunk.FilePath != nil {
		return nil, ci, cm, fmt.Errorf("nyi: data is in another file: '%s'", *chunk.FilePath)
	}
	if chunk.MetaData == nil {
		return nil, ci, cm, fmt.Errorf("missing meta data for Column %c", col.Index())
	}
	if typ := *col.Element().Type; chunk.MetaData.Type != typ {
		return nil, ci, cm, fmt.Errorf("wrong type in Column chunk metadata, expected %s was %s", typ, chunk.MetaData.Type)
	}
	md := chunk.MetaData
	start := md.DataPageOffset
	if md.DictionaryPageOffset != nil {
		start = *md.DictionaryPageOffset
	}
	buf := make([]byte, md.TotalCompressedSize)
	if _, err := f.reader.Seek(start, io.SeekStart); err != nil {
		return nil, ci, cm, err
	}
	n, err := io.ReadFull(f.reader, buf)
	if err != nil && err != io.ErrUnexpectedEOF {
		return nil, ci, cm, err
	}
	el := col.Element()
	ci = gpudecode.ColumnInfo{
		PhysicalType: int(*el.Type), MaxDef: int(col.MaxDefinitionLevel()), MaxRep: int(col.MaxRepetitionLevel()),
	}
	if el.TypeLength != nil {
		ci.TypeLength = int(*el.TypeLength)
	}
	cm = gpudecode.ChunkMeta{
		PhysicalType: int(md.Type), Codec: int(md.Codec), NumValues: md.NumValues,
		TotalCompressedSize: md.TotalCompressedSize, DataPageOffset: md.DataPageOffset - start,
		DictionaryPageOffset: -1, HasFilePath: false,
	}
	if md.DictionaryPageOffset != nil {
		cm.DictionaryPageOffset = 0
	}
	return buf[:n], ci, cm, nil
}

// readRowGroupDataGPU replaces readRowGroupData (chunk_reader.go:375-404) when the reader has a
// GPU: every selected column chunk of the row group goes into ONE batch (one set of kernel
// launches for all its pages), decoded once; then the columns are handed their pages in column
// order, returning the first error where the reference's loop would meet it: a readChunk /
// readPages error (headers, CRC, decompression) for that column's turn; a readValues error only
// from its page on (the pages before it read normally).
func (f *FileReader) readRowGroupDataGPU(ctx context.Context) error {
	rowGroup := f.meta.RowGroups[f.rowGroupPosition-1]
	dataCols := f.schemaReader.Columns()

	f.schemaReader.resetData()
	f.schemaReader.setNumRecords(rowGroup.NumRows)
	b, err := gpudecode.NewBatch(f.gpu)
	if err != nil {
		return err
	}
	defer b.Close()
	type planned struct {
		col *Column
		id  int32
		err error // readChunk error of this column (returned at its turn)
	}
	var cols []planned
	for _, c := range dataCols {
		idx := c.Index()
		if len(rowGroup.Columns) <= idx {
			cols = append(cols, planned{col: c, err: fmt.Errorf("column index %d is out of bounds", idx)})
			break
		}
		chunk := rowGroup.Columns[idx]
		if !f.schemaReader.isSelectedByPath(c.path) {
			if err := f.skipChunk(c, chunk); err != nil {
				cols = append(cols, planned{col: c, err: err})
				break
			}
			c.data.skipped = true
			continue
		}
		buf, ci, cm, err := f.gpuChunkInput(c, chunk)
		if err != nil {
			cols = append(cols, planned{col: c, err: err})
			break
		}
		id, err := b.AddChunk(buf, ci, cm, f.schemaReader.validateCRC)
		cols = append(cols, planned{col: c, id: id, err: err})
		if err != nil {
			break // readPages failed on the host: the reference returns before later columns
		}
	}
	if err := b.Decode(); err != nil {
		return err
	}
	_ = b.Sync()
	for _, p := range cols {
		if p.err != nil {
			return p.err
		}
		res, rerr := b.Result(p.id)
		if rerr != nil && gpudecode.ReadPagesError(rerr) {
			return rerr // decompression / CRC: readPages fails before any value is read
		}
		failPage := -1
		var failErr error
		if rerr != nil {
			failPage, failErr = rerr.(*gpudecode.DecodeError).Page, fmt.Errorf("read values from page failed: %w", rerr)
		}
		useDict := res != nil && res.DictionaryPage
		if err := readPageData(p.col, gpuPages(p.col, res, failPage, failErr), useDict); err != nil {
			return err
		}
	}
	return nil
}

// gpuPages splits a decoded chunk into per-page readers; pages from the failing
// one on return its error (the reference never reads past it). For a failing
// chunk `res` holds the decoded pages before the failing page.
func gpuPages(col *Column, res *gpudecode.Chunk, failPage int, failErr error) []pageReader {
	if res == nil {
		return []pageReader{&gpuPageReader{err: failErr, n: 1}}
	}
	maxD, maxR := col.MaxDefinitionLevel(), col.MaxRepetitionLevel()
	pages := make([]pageReader, 0, len(res.Pages))
	for k, pg := range res.Pages {
		p := &gpuPageReader{n: int32(pg.SlotCount)}
		if failPage >= 0 && k >= failPage {
			p.err = failErr
			pages = append(pages, p)
			continue
		}
		p.dLevel, p.rLevel = &packedArray{}, &packedArray{}
		p.dLevel.reset(bits.Len16(maxD))
		p.rLevel.reset(bits.Len16(maxR))
		for s := pg.SlotFirst; s < pg.SlotFirst+pg.SlotCount; s++ {
			p.dLevel.appendSingle(res.DefLevel(s))
			p.rLevel.appendSingle(res.RepLevel(s))
		}
		p.values = make([]interface{}, pg.ValueCount)
		for i := range p.values {
			p.values[i] = gpuValue(res, pg.ValueFirst+int64(i))
		}
		pages = append(pages, p)
	}
	return pages
}

// gpuValue boxes value v the way the CPU decoders do (type_*.go): raw bits for
// floats (type_float.go:28, type_double.go:28), [12]byte INT96, []byte arrays.
func gpuValue(res *gpudecode.Chunk, v int64) interface{} {
	w := int64(res.ValueWidth)
	switch parquet.Type(res.PhysicalType) {
	case parquet.Type_BOOLEAN:
		return res.Values[v] != 0
	case parquet.Type_INT32:
		return int32(binary.LittleEndian.Uint32(res.Values[v*4:]))
	case parquet.Type_INT64:
		return int64(binary.LittleEndian.Uint64(res.Values[v*8:]))
	case parquet.Type_FLOAT:
		return math.Float32frombits(binary.LittleEndian.Uint32(res.Values[v*4:]))
	case parquet.Type_DOUBLE:
		return math.Float64frombits(binary.LittleEndian.Uint64(res.Values[v*8:]))
	case parquet.Type_INT96:
		var x [12]byte
		copy(x[:], res.Values[v*12:v*12+12])
		return x
	case parquet.Type_FIXED_LEN_BYTE_ARRAY:
		if w > 0 {
			return append([]byte(nil), res.Values[v*w:(v+1)*w]...)
		}
	}
	return append([]byte(nil), res.Payload[res.Offsets[v]:res.Offsets[v+1]]...)
}
