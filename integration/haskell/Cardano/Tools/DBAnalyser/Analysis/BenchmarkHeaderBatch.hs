{-# LANGUAGE BangPatterns        #-}
{-# LANGUAGE RankNTypes          #-}
{-# LANGUAGE NamedFieldPuns      #-}
{-# LANGUAGE ScopedTypeVariables #-}

-- | A db-analyser analysis beside 'BenchmarkLedgerOps' (Analysis.hs:75-88, :479-607):
-- header revalidation of a Praos (Babbage/Conway) ImmutableDB in per-epoch batches on the
-- GPU through 'Ouroboros.Consensus.Protocol.Praos.Batch' (Storable vectors in and out), timed
-- per epoch on the monotonic wall clock, one line per epoch:
--
--   epoch  headers  validated  stop_verdict  ms  headers/s
--
-- A maintainer wires it in as one more 'AnalysisName' constructor
-- (@BenchmarkHeaderBatch (Maybe FilePath) Int@: output file, device) and one more
-- equation of runAnalysis (Analysis.hs:108-123).  The stream is the same
-- 'processAllImmutableDB' loop (Analysis.hs:815-847) with 'GetRawHeader' as the block
-- component, so the bytes the GPU decodes are exactly the stored header spans the
-- secondary index gives (Secondary.hs:93-128).  Shipped as source (no GHC here); the
-- ABI calls it makes are replayed from C by integration/c/ffi_harness.c.
module Cardano.Tools.DBAnalyser.Analysis.BenchmarkHeaderBatch
  ( benchmarkHeaderBatch
  , EpochBatchEnv (..)
  ) where

import           Control.Monad (unless, when)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Lazy as BSL
import           Data.IORef
import qualified Data.Vector.Storable as VS
import qualified Data.Vector.Storable.Mutable as VSM
import           Data.Word (Word16, Word32, Word64, Word8)
import           GHC.Clock (getMonotonicTimeNSec)
import qualified System.IO as IO
import           Text.Printf (hPrintf)

import           Ouroboros.Consensus.Protocol.Praos.Batch

-- | What the analysis needs besides the stream: the epoch layout and stability window
-- (praosParams / EpochInfo), the ledger view (PoolDistr, envelope limits) installed per
-- epoch, the protocol parameters, and the genesis PraosState (CBOR).
data EpochBatchEnv = EpochBatchEnv
  { ebEpochInfo   :: (Word64, Word64, Word64, Word64)   -- base slot, base epoch, length, window
  , ebEnvLimits   :: (Word64, Word64, Word64, Word64)   -- maxMajorPV, pvMajor, maxHeaderSize, maxBodySize
  , ebPools       :: Word64 -> [(BS.ByteString, BS.ByteString, Integer)]   -- PoolDistr of an epoch
  , ebParams      :: PraosParamsC
  , ebStateCbor   :: BS.ByteString
  , ebDevice      :: Int
  }

-- | @benchmarkHeaderBatch out env stream@: @stream@ is the analysis' processAll over the
-- ImmutableDB with 'GetRawHeader' (slot and raw header bytes per block), folded here into
-- per-epoch batches.
benchmarkHeaderBatch
  :: Maybe FilePath
  -> EpochBatchEnv
  -> (forall st. st -> (st -> (Word64, BSL.ByteString) -> IO (Bool, st)) -> IO st)
  -> IO ()
benchmarkHeaderBatch mOut EpochBatchEnv {ebEpochInfo, ebEnvLimits, ebPools, ebParams, ebStateCbor, ebDevice}
                     stream =
  withOut mOut $ \h -> withPraosBatchCtx ebDevice $ \ctx -> do
    IO.hPutStrLn h "epoch\theaders\tvalidated\tstop_verdict\tms\theaders/s"
    stRef <- newIORef ebStateCbor
    tipRef <- newIORef Nothing
    let (base, baseNo, len, _) = ebEpochInfo
        epochOf s = baseNo + (s - base) `div` len
        -- one epoch's batch: tick, install the ledger view, validate, report
        flush _ [] = pure True
        flush e hdrsRev = do
          st <- readIORef stRef
          tip <- readIORef tipRef
          let hdrs = reverse hdrsRev
              firstSlot = fst (head hdrs)
              raws = map snd hdrs
              n = length hdrs
              arena = BS.concat raws
              lens = VS.fromListN n (map (fromIntegral . BS.length) raws) :: VS.Vector Word32
              offs = VS.prescanl' (+) 0 (VS.map fromIntegral lens)
          eta <- praosTickedEpochNonce st ebEpochInfo firstSlot
          praosSetEpoch ctx eta (ebPools e) ebParams
          verdicts <- VSM.new n :: IO (VSM.IOVector Word8)
          bits <- VSM.new n :: IO (VSM.IOVector Word16)
          -- wall clock around the batch (the foreign call is safe: mutator time would not
          -- count the time the GPU spends)
          t0 <- getMonotonicTimeNSec
          !r <- praosValidateHeaderSpans ctx ebEpochInfo ebEnvLimits tip st arena offs lens verdicts bits
          t1 <- getMonotonicTimeNSec
          let ms = fromIntegral (t1 - t0) / 1e6 :: Double
              stopped = srChainStop r < n
          verdict <- if stopped then VSM.read verdicts (srChainStop r) else pure 0
          hPrintf h "%d\t%d\t%d\t%d\t%.3f\t%.0f\n" e n (srChainStop r) verdict ms
                  (fromIntegral n / max 1e-9 (ms / 1e3))
          writeIORef stRef (srState r)
          writeIORef tipRef (srTip r)
          pure (not stopped)          -- the reference stops at the first invalid header
    (e, acc, ok) <- stream (0, [], True) $ \(e, acc, ok) (slot, raw) -> do
      let e' = epochOf slot
          hdr = (slot, BSL.toStrict raw)
      if null acc || e' == e
        then pure (True, (e', hdr : acc, ok))
        else do
          ok' <- flush e acc
          pure (ok', (e', [hdr], ok'))
    when ok $ do
      _ <- flush e acc
      pure ()
    unless ok $ IO.hPutStrLn h "# stopped at the first invalid header"
  where
    withOut (Just f) k = IO.withFile f IO.WriteMode k
    withOut Nothing k = k IO.stdout
