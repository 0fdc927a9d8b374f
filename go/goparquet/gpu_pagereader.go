// gpu_pagereader.go — the in-package half of the MI355X decode path for
// github.com/fraugster/parquet-go (package goparquet).
//
// pageReader / valuesDecoder / levelDecoder are unexported (interfaces.go:11-39,
// hybrid_decoder.go:16-27), so only a file inside package goparquet can stand
// behind them. Copy this file next to chunk_reader.go and apply the three-line
// hook of INTEGRATION.md (a `gpu` field on FileReader / fileReaderOptions and a
// call at the top of readChunk). With WithGPUDecoder(ctx) a FileReader decodes
// each selected column chunk on the GPU in one batch (every page, levels and
// values) and hands ColumnStore.readNextPage (data_store.go:236-260) one
// gpuPageReader per data page, exactly the (values, dLevel, rLevel) triple the
// CPU pageReaders return, including the error of the first failing page.
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

// readChunkGPU replaces readChunk + readPages (chunk_reader.go:182-362) for one chunk.
func (f *FileReader) readChunkGPU(ctx context.Context, col *Column, chunk *parquet.ColumnChunk) ([]pageReader, bool, error) {
	md := chunk.MetaData
	start := md.DataPageOffset
	if md.DictionaryPageOffset != nil {
		start = *md.DictionaryPageOffset
	}
	buf := make([]byte, md.TotalCompressedSize)
	if _, err := f.reader.Seek(start, io.SeekStart); err != nil {
		return nil, false, err
	}
	n, err := io.ReadFull(f.reader, buf)
	if err != nil && err != io.ErrUnexpectedEOF {
		return nil, false, err
	}
	buf = buf[:n]
	el := col.Element()
	ci := gpudecode.ColumnInfo{
		PhysicalType: int(*el.Type), MaxDef: int(col.MaxDefinitionLevel()), MaxRep: int(col.MaxRepetitionLevel()),
	}
	if el.TypeLength != nil {
		ci.TypeLength = int(*el.TypeLength)
	}
	cm := gpudecode.ChunkMeta{
		PhysicalType: int(md.Type), Codec: int(md.Codec), NumValues: md.NumValues,
		TotalCompressedSize: md.TotalCompressedSize, DataPageOffset: md.DataPageOffset - start,
		DictionaryPageOffset: -1, HasFilePath: chunk.FilePath != nil,
	}
	if md.DictionaryPageOffset != nil {
		cm.DictionaryPageOffset = 0
	}
	b, err := gpudecode.NewBatch(f.gpu)
	if err != nil {
		return nil, false, err
	}
	defer b.Close()
	id, err := b.AddChunk(buf, ci, cm, f.schemaReader.validateCRC)
	if err != nil {
		return nil, false, err // readChunk / readPages error (page headers, dictionary page)
	}
	if err := b.Decode(); err != nil {
		return nil, false, err
	}
	_ = b.Sync()
	failPage := -1
	var failErr error
	if err := b.Status(id); err != nil {
		de, ok := err.(*gpudecode.DecodeError)
		if !ok || de.Page < 0 {
			return nil, false, err
		}
		failPage, failErr = de.Page, fmt.Errorf("read values from page failed: %w", err)
	}
	res, rerr := b.Result(id)
	if rerr != nil && failPage < 0 {
		return nil, false, rerr
	}
	return gpuPages(col, res, failPage, failErr), md.DictionaryPageOffset != nil, nil
}

// gpuPages splits a decoded chunk into per-page readers; pages from the failing
// one on return its error (the reference never reads past it).
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
